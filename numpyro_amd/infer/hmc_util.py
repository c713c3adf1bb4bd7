"""numpyro.infer.hmc_util's kinetic-energy helpers (hmc_util.py:1183-1220), for callers that
pass the Euclidean kinetic energy explicitly (``NUTS(model, kinetic_fn=euclidean_kinetic_energy)``)
or evaluate it on a state.  The device integrates exactly this kinetic energy (the leapfrog's
momentum step uses its gradient, ``euclidean_kinetic_grad``); any other ``kinetic_fn`` is refused
by ``HMC`` / ``NUTS``: a user function of the momentum would have to be compiled into the leaf."""
import torch

__all__ = ["euclidean_kinetic_energy", "euclidean_kinetic_grad"]


def _ravel(r):
    """ravel_pytree (jax.flatten_util): the flat vector and the function mapping a flat vector back
    to r's structure.  A plain dict flattens by sorted key, an OrderedDict in insertion order (as
    jax's pytree registry does), tuples / lists in order."""
    from collections import OrderedDict

    if isinstance(r, dict):
        keys = list(r) if isinstance(r, OrderedDict) else sorted(r)
        leaves = [torch.as_tensor(r[k]) for k in keys]
        flat = torch.cat([v.reshape(-1) for v in leaves])

        def unravel(v):
            out, o = OrderedDict() if isinstance(r, OrderedDict) else {}, 0
            for k, leaf in zip(keys, leaves):
                n = leaf.numel()
                out[k] = v[o:o + n].reshape(leaf.shape)
                o += n
            return out
        return flat, unravel
    if isinstance(r, (tuple, list)):
        leaves = [torch.as_tensor(v) for v in r]
        flat = torch.cat([v.reshape(-1) for v in leaves])

        def unravel(v):
            out, o = [], 0
            for leaf in leaves:
                out.append(v[o:o + leaf.numel()].reshape(leaf.shape))
                o += leaf.numel()
            return type(r)(out)
        return flat, unravel
    t = torch.as_tensor(r)
    return t.reshape(-1), lambda v: v.reshape(t.shape)


def euclidean_kinetic_energy(inverse_mass_matrix, r):
    """0.5 r^T M^-1 r (hmc_util.py:1183-1200): M^-1 a matrix [D, D], a diagonal [D], or a dict
    {site-name tuple: block} of a structured mass (the blocks' momenta taken in the tuple's order)."""
    if isinstance(inverse_mass_matrix, dict):
        ke = 0.0
        for names, block in inverse_mass_matrix.items():
            ke = ke + euclidean_kinetic_energy(block, tuple(r[k] for k in names))
        return ke
    r, _ = _ravel(r)
    imm = torch.as_tensor(inverse_mass_matrix, dtype=r.dtype, device=r.device)
    if imm.dim() not in (1, 2):
        raise ValueError("inverse_mass_matrix should have 1 or 2 dimensions.")
    v = imm @ r if imm.dim() == 2 else imm * r
    return 0.5 * torch.dot(v, r)


def euclidean_kinetic_grad(inverse_mass_matrix, r):
    """dK/dr = M^-1 r in r's own structure (hmc_util.py:1203-1223): the flat product unraveled
    like r (ravel_pytree / unravel_fn); for a dict of site-group blocks a {site: grad} dict, each
    block's momenta taken in the group's order (the reference's OrderedDict r_block)."""
    from collections import OrderedDict

    if isinstance(inverse_mass_matrix, dict):
        r_grad = {}
        for names, block in inverse_mass_matrix.items():
            r_grad.update(euclidean_kinetic_grad(block, OrderedDict((k, r[k]) for k in names)))
        return r_grad
    flat, unravel = _ravel(r)
    imm = torch.as_tensor(inverse_mass_matrix, dtype=flat.dtype, device=flat.device)
    if imm.dim() not in (1, 2):
        raise ValueError("inverse_mass_matrix should have 1 or 2 dimensions.")
    return unravel(imm @ flat if imm.dim() == 2 else imm * flat)


euclidean_kinetic_energy._kinetic_grad = euclidean_kinetic_grad
