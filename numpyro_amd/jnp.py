"""The array functions the reference's example models call on jax.numpy (matmul, dot, tanh,
exp, sqrt, zeros, ones, shape), working on NumPy / torch arrays and on the symbolic values of
latent sites while the model front end traces a model (numpyro_amd/frontend.py).  Write
``from numpyro_amd import jnp`` where a numpyro model has ``import jax.numpy as jnp``."""
from __future__ import annotations

import numpy as np


class Sym:
    """Symbolic value in a traced model: a latent site or an operation on symbolic values.
    ``op``: "latent" (args = (name,)), or an operation name with argument values (Sym,
    numbers or arrays)."""

    __array_priority__ = 1000  # NumPy arrays defer binary operators to Sym

    def __init__(self, op, args, shape):
        self.op, self.args, self.shape = op, tuple(args), tuple(shape)

    # arithmetic builds expressions
    def _bin(self, op, other, reverse=False):
        a, b = (other, self) if reverse else (self, other)
        return Sym(op, (a, b), np.broadcast_shapes(shape_of(a), shape_of(b)))

    def __add__(self, o): return self._bin("add", o)
    def __radd__(self, o): return self._bin("add", o, True)
    def __sub__(self, o): return self._bin("sub", o)
    def __rsub__(self, o): return self._bin("sub", o, True)
    def __mul__(self, o): return self._bin("mul", o)
    def __rmul__(self, o): return self._bin("mul", o, True)
    def __truediv__(self, o): return self._bin("div", o)
    def __rtruediv__(self, o): return self._bin("div", o, True)
    def __neg__(self): return Sym("neg", (self,), self.shape)
    def __matmul__(self, o): return matmul(self, o)
    def __rmatmul__(self, o): return matmul(o, self)
    def __pow__(self, o): return self._bin("pow", o)

    def __repr__(self):
        if self.op == "latent":
            return f"<{self.args[0]}>"
        return f"{self.op}({', '.join(repr(a) if isinstance(a, Sym) else type(a).__name__ for a in self.args)})"


def shape_of(x):
    if isinstance(x, Sym):
        return x.shape
    if hasattr(x, "shape"):
        return tuple(x.shape)
    return np.shape(x)


def _unary(name, fn):
    def f(x):
        if isinstance(x, Sym):
            return Sym(name, (x,), x.shape)
        return fn(np.asarray(x) if not hasattr(x, "cpu") else x.cpu().numpy())
    f.__name__ = name
    return f


tanh = _unary("tanh", np.tanh)
exp = _unary("exp", np.exp)
sqrt = _unary("sqrt", np.sqrt)
log = _unary("log", np.log)


def matmul(a, b):
    if isinstance(a, Sym) or isinstance(b, Sym):
        sa, sb = shape_of(a), shape_of(b)
        out = sa[:-1] + sb[1:] if len(sb) > 1 else sa[:-1]
        return Sym("matmul", (a, b), out)
    return np.matmul(np.asarray(a), np.asarray(b))


dot = matmul


def zeros(shape, dtype=None):
    return np.zeros(shape, np.float32)


def ones(shape, dtype=None):
    return np.ones(shape, np.float32)


def shape(x):
    return shape_of(x)
