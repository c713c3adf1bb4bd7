"""Distribution descriptors of the hot path (numpyro/distributions), for models written against
numpyro's API and run through the model front end (numpyro_amd/frontend.py).

They hold their parameters (numbers, arrays, or symbolic values of latent sites while a model
is traced) and shapes; the arithmetic runs in the fused kernels the front end maps a traced
model onto, so there is no log_prob here.  Names and signatures follow numpyro:
Normal (continuous.py:2171), HalfCauchy (:700), Exponential (:455), Gamma (:490), StudentT
(:2344), Bernoulli / BernoulliLogits (discrete.py:108-139), GaussianRandomWalk (continuous.py:
658), MultivariateNormal (:1487); ``.to_event`` / ``.expand`` (distribution.py:377-420).
"""
from __future__ import annotations

import numpy as np

from .jnp import shape_of


def _bshape(*params):
    shapes = [shape_of(p) for p in params if p is not None]
    return tuple(np.broadcast_shapes(*shapes)) if shapes else ()


class Distribution:
    support = "real"

    def __init__(self, batch_shape=(), event_shape=()):
        self.batch_shape = tuple(batch_shape)
        self.event_shape = tuple(event_shape)

    @property
    def shape(self):
        return self.batch_shape + self.event_shape

    def to_event(self, reinterpreted_batch_ndims=None):
        n = len(self.batch_shape) if reinterpreted_batch_ndims is None else int(reinterpreted_batch_ndims)
        return Independent(self, n)

    def expand(self, batch_shape):
        return ExpandedDistribution(self, tuple(batch_shape))

    def params(self):
        return {}

    def __repr__(self):
        return f"{type(self).__name__}(batch_shape={self.batch_shape}, event_shape={self.event_shape})"


class Independent(Distribution):
    def __init__(self, base, reinterpreted_batch_ndims):
        n = reinterpreted_batch_ndims
        bs = base.batch_shape
        super().__init__(bs[:len(bs) - n], bs[len(bs) - n:] + base.event_shape)
        self.base_dist = base
        self.support = base.support

    def params(self):
        return self.base_dist.params()


class ExpandedDistribution(Distribution):
    def __init__(self, base, batch_shape):
        super().__init__(batch_shape, base.event_shape)
        self.base_dist = base
        self.support = base.support

    def params(self):
        return self.base_dist.params()


class Normal(Distribution):
    def __init__(self, loc=0.0, scale=1.0):
        super().__init__(_bshape(loc, scale))
        self.loc, self.scale = loc, scale

    def params(self):
        return {"loc": self.loc, "scale": self.scale}


class HalfCauchy(Distribution):
    support = "positive"

    def __init__(self, scale=1.0):
        super().__init__(_bshape(scale))
        self.scale = scale

    def params(self):
        return {"scale": self.scale}


class Exponential(Distribution):
    support = "positive"

    def __init__(self, rate=1.0):
        super().__init__(_bshape(rate))
        self.rate = rate

    def params(self):
        return {"rate": self.rate}


class Gamma(Distribution):
    support = "positive"

    def __init__(self, concentration, rate=1.0):
        super().__init__(_bshape(concentration, rate))
        self.concentration, self.rate = concentration, rate

    def params(self):
        return {"concentration": self.concentration, "rate": self.rate}


class StudentT(Distribution):
    def __init__(self, df, loc=0.0, scale=1.0):
        super().__init__(_bshape(df, loc, scale))
        self.df, self.loc, self.scale = df, loc, scale

    def params(self):
        return {"df": self.df, "loc": self.loc, "scale": self.scale}


class BernoulliLogits(Distribution):
    support = "boolean"

    def __init__(self, logits):
        super().__init__(_bshape(logits))
        self.logits = logits

    def params(self):
        return {"logits": self.logits}


class BernoulliProbs(Distribution):
    support = "boolean"

    def __init__(self, probs):
        super().__init__(_bshape(probs))
        self.probs = probs

    def params(self):
        return {"probs": self.probs}


def Bernoulli(probs=None, logits=None):
    """numpyro/distributions/discrete.py:142-151 dispatch on probs / logits."""
    if (probs is None) == (logits is None):
        raise ValueError("One of `probs` or `logits` must be specified.")
    return BernoulliLogits(logits) if logits is not None else BernoulliProbs(probs)


class GaussianRandomWalk(Distribution):
    def __init__(self, scale=1.0, num_steps=1):
        super().__init__(_bshape(scale), (int(num_steps),))
        self.scale, self.num_steps = scale, int(num_steps)

    def params(self):
        return {"scale": self.scale, "num_steps": self.num_steps}


class MultivariateNormal(Distribution):
    def __init__(self, loc=0.0, covariance_matrix=None, precision_matrix=None, scale_tril=None):
        if scale_tril is not None:
            st = np.asarray(scale_tril, np.float64)
            covariance_matrix = st @ st.T
        mats = [m for m in (covariance_matrix, precision_matrix) if m is not None]
        if len(mats) != 1:
            raise ValueError("One of `covariance_matrix`, `precision_matrix`, `scale_tril` must be specified.")
        d = shape_of(mats[0])[-1]
        super().__init__((), (d,))
        self.loc = loc
        self.covariance_matrix, self.precision_matrix = covariance_matrix, precision_matrix

    def params(self):
        return {"loc": self.loc, "covariance_matrix": self.covariance_matrix,
                "precision_matrix": self.precision_matrix}
