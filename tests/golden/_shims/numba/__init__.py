"""Identity stand-in for numba (absent from this image; no network).

Used ONLY by tests/golden/gen_golden.py, in this container, to import the
read-only reference so it can produce golden vectors.  `@njit` / `@jit` bodies
then run as plain CPython/numpy, which is semantically the same program
(numba only JIT-compiles); see SURVEY.md §8c "Semantics caveat of the shim".
"""


def _identity_decorator(*args, **kwargs):
    if len(args) == 1 and callable(args[0]) and not kwargs:
        return args[0]

    def wrap(fn):
        return fn
    return wrap


njit = _identity_decorator
jit = _identity_decorator
