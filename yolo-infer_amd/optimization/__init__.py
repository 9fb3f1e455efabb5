"""Model optimisation plugins (the reference's `optimization/` package): the PTQ int8 path of the MI355X runtime."""
