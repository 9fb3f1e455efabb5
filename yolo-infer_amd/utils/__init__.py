"""Host-side helpers of the reference's `utils/` that the predict path's consumers call."""
