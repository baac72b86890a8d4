"""The reference's optional numba shim (speedup.py:2-19); the MI355X build needs no JIT."""


def jit(*args, **kwargs):
    if args and callable(args[0]):
        return args[0]
    return lambda f: f
