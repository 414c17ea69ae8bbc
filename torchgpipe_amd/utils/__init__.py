"""Framework utilities: RNG tapes, tracing, checkpoint (state) I/O, profiling."""
