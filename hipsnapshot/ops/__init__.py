"""Native ops: ctypes bindings to the HIP data plane and the C++ I/O engine."""
