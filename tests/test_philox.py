"""Philox4x32-10 known-answer tests (Random123 kat_vectors) for the oracle and the device."""
import numpy as np
import pytest

from oracle.philox import philox4x32_10, rng, u01

KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


@pytest.mark.parametrize("ctr,key,expected", KAT)
def test_oracle_philox_kat(ctr, key, expected):
    assert list(philox4x32_10(ctr, key)) == expected


def test_oracle_uniform_range():
    x = rng(123, np.arange(1000), 0, 4, 0, 0)[:, 0]
    u = u01(x)
    assert u.dtype == np.float32
    assert (u >= 0).all() and (u < 1).all()
    assert abs(u.mean() - 0.5) < 0.05


@pytest.mark.gpu
def test_device_philox_matches_oracle(device):
    import torch
    from numpyro_amd import native

    rs = np.random.RandomState(0)
    ctr_key = np.concatenate(
        [np.array([c + k for c, k, _ in KAT], dtype=np.uint64).astype(np.uint32),
         rs.randint(0, 2**32, size=(253, 6), dtype=np.uint64).astype(np.uint32)])
    n = ctr_key.shape[0]
    d_in = torch.from_numpy(ctr_key.view(np.int32)).to(device)
    d_out = torch.zeros(n * 4, dtype=torch.int32, device=device)
    native.check(native.lib().nmx_selftest_philox(native.ptr(d_in), native.ptr(d_out), n,
                                                   native.stream_ptr()))
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.uint32).reshape(n, 4)
    exp = philox4x32_10(ctr_key[:, :4], ctr_key[:, 4:])
    np.testing.assert_array_equal(got, exp)
    for i, (_, _, e) in enumerate(KAT):
        assert list(got[i]) == e
