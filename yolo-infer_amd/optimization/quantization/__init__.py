from .quantizers import PostTrainingQuantizer, create_quantizer  # noqa: F401
