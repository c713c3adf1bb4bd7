"""The reference's example models written against numpyro's API with numpyro_amd's
primitives (verbatim structure of examples/covtype.py:66-71, README.md:47-55,
examples/funnel.py:44-49, examples/stochastic_volatility.py:57-65, examples/bnn.py:43-74)."""
import numpyro_amd as numpyro
from numpyro_amd import distributions as dist
from numpyro_amd import jnp


def covtype_model(data, labels):
    dim = data.shape[1]
    coefs = numpyro.sample("coefs", dist.Normal(jnp.zeros(dim), jnp.ones(dim)))
    logits = jnp.dot(data, coefs)
    return numpyro.sample("obs", dist.Bernoulli(logits=logits), obs=labels)


def eight_schools(J, sigma, y=None):
    mu = numpyro.sample("mu", dist.Normal(0, 5))
    tau = numpyro.sample("tau", dist.HalfCauchy(5))
    with numpyro.plate("J", J):
        theta = numpyro.sample("theta", dist.Normal(mu, tau))
        numpyro.sample("obs", dist.Normal(theta, sigma), obs=y)


def funnel(dim=10):
    y = numpyro.sample("y", dist.Normal(0, 3))
    numpyro.sample("x", dist.Normal(jnp.zeros(dim - 1), jnp.exp(y / 2)))


funnel_reparam = numpyro.reparam(funnel, config={"x": numpyro.LocScaleReparam(0)})


def stochastic_volatility(returns):
    step_size = numpyro.sample("sigma", dist.Exponential(50.0))
    s = numpyro.sample("s", dist.GaussianRandomWalk(scale=step_size, num_steps=jnp.shape(returns)[0]))
    nu = numpyro.sample("nu", dist.Exponential(0.1))
    return numpyro.sample("r", dist.StudentT(df=nu, loc=0.0, scale=jnp.exp(s)), obs=returns)


def nonlin(x):
    return jnp.tanh(x)


def bnn(X, Y, D_H, D_Y=1):
    N, D_X = X.shape
    w1 = numpyro.sample("w1", dist.Normal(jnp.zeros((D_X, D_H)), jnp.ones((D_X, D_H))))
    z1 = nonlin(jnp.matmul(X, w1))
    w2 = numpyro.sample("w2", dist.Normal(jnp.zeros((D_H, D_H)), jnp.ones((D_H, D_H))))
    z2 = nonlin(jnp.matmul(z1, w2))
    w3 = numpyro.sample("w3", dist.Normal(jnp.zeros((D_H, D_Y)), jnp.ones((D_H, D_Y))))
    z3 = jnp.matmul(z2, w3)
    prec_obs = numpyro.sample("prec_obs", dist.Gamma(3.0, 1.0))
    sigma_obs = 1.0 / jnp.sqrt(prec_obs)
    with numpyro.plate("data", N):
        numpyro.sample("Y", dist.Normal(z3, sigma_obs).to_event(1), obs=Y)
