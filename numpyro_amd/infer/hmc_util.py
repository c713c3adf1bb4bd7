"""numpyro.infer.hmc_util's kinetic-energy helpers (hmc_util.py:1183-1220), for callers that
pass the Euclidean kinetic energy explicitly (``NUTS(model, kinetic_fn=euclidean_kinetic_energy)``)
or evaluate it on a state.  The device integrates exactly this kinetic energy (the leapfrog's
momentum step uses its gradient, ``euclidean_kinetic_grad``); any other ``kinetic_fn`` is refused
by ``HMC`` / ``NUTS``: a user function of the momentum would have to be compiled into the leaf."""
import torch

__all__ = ["euclidean_kinetic_energy", "euclidean_kinetic_grad"]


def _ravel(r):
    """ravel_pytree order: dict sites by sorted name, tuples / lists in order, then flattened."""
    if isinstance(r, dict):
        return torch.cat([torch.as_tensor(r[k]).reshape(-1) for k in sorted(r)])
    if isinstance(r, (tuple, list)):
        return torch.cat([torch.as_tensor(v).reshape(-1) for v in r])
    return torch.as_tensor(r).reshape(-1)


def euclidean_kinetic_energy(inverse_mass_matrix, r):
    """0.5 r^T M^-1 r (hmc_util.py:1183-1200): M^-1 a matrix [D, D], a diagonal [D], or a dict
    {site-name tuple: block} of a structured mass (the blocks' momenta taken in the tuple's order)."""
    if isinstance(inverse_mass_matrix, dict):
        ke = 0.0
        for names, block in inverse_mass_matrix.items():
            ke = ke + euclidean_kinetic_energy(block, tuple(r[k] for k in names))
        return ke
    r = _ravel(r)
    imm = torch.as_tensor(inverse_mass_matrix, dtype=r.dtype, device=r.device)
    v = imm @ r if imm.dim() == 2 else imm * r
    return 0.5 * torch.dot(v, r)


def euclidean_kinetic_grad(inverse_mass_matrix, r):
    """dK/dr = M^-1 r (hmc_util.py:1203-1220), raveled."""
    if isinstance(inverse_mass_matrix, dict):
        return torch.cat([euclidean_kinetic_grad(b, tuple(r[k] for k in names))
                          for names, b in inverse_mass_matrix.items()])
    r = _ravel(r)
    imm = torch.as_tensor(inverse_mass_matrix, dtype=r.dtype, device=r.device)
    return imm @ r if imm.dim() == 2 else imm * r


euclidean_kinetic_energy._kinetic_grad = euclidean_kinetic_grad
