"""Test infrastructure: numpy restatement of the ENGINE's reparameterisation noise.

The reference draws torch::randn_like (unseeded), which no two runs share; the engine
instead keys every draw by (seed, step, global row, latent) through Philox4x32-10 + Box-Muller
(mm-vae_amd/csrc/common.hpp philox4x32_10 / philox_normal) so a data-parallel shard draws the
single-GPU noise.  This module restates that generator so an oracle loop (oracle/nb_oracle.py,
the reference's op sequence on ATen CPU) can be fed the very noise a CLI run used — tests only.

The integer rounds are exact; the device's Box-Muller runs on v_log / v_sqrt / v_sin / v_cos
(approximate to ~1 ulp), this one in float64 — agreement ~1e-6 relative (tests/test_gpu_host.py).
"""
import numpy as np

_M32 = np.uint64(0xFFFFFFFF)


def _philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(v, np.uint64) & _M32 for v in (c0, c1, c2, c3))
    k0 = np.uint64(k0) & _M32
    k1 = np.uint64(k1) & _M32
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _M32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _M32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + np.uint64(0x9E3779B9)) & _M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & _M32
    return c0, c1, c2, c3


def philox_normal(seed, step, rows, ks):
    """eps(seed, step, row, k) for arrays rows [n], ks [m] -> [n, m] float32."""
    seed, step = int(seed), int(step)
    rows = np.asarray(rows, np.uint64)[:, None]
    ks = np.asarray(ks, np.uint64)[None, :]
    c0 = np.broadcast_to(ks >> np.uint64(1), (rows.shape[0], ks.shape[1]))
    c1 = np.broadcast_to(rows & _M32, c0.shape)
    c2 = np.broadcast_to((rows >> np.uint64(32)) ^ np.uint64(step & 0xFFFFFFFF), c0.shape)
    c3 = np.full(c0.shape, np.uint64((step >> 32) & 0xFFFFFFFF))
    r0, r1, _, _ = _philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    u1 = ((r0 >> np.uint64(8)) + np.uint64(1)).astype(np.float32) * np.float32(1.0 / 16777217.0)  # (0, 1]
    u2 = (r1 >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)                   # [0, 1)
    r = np.sqrt(-2.0 * np.log(u1.astype(np.float64)))
    ang = 2.0 * np.pi * u2.astype(np.float64)
    odd = (np.broadcast_to(ks, c0.shape) & np.uint64(1)).astype(bool)
    return (r * np.where(odd, np.sin(ang), np.cos(ang))).astype(np.float32)


def nb_step_noise(seed, step, B, K, R=1, row_offset=0):
    """The NB step's (eps_mu [B, K], eps_nu [B, R]): latent k keyed k, overdispersion r keyed
    NU_LANE + r = 2^31 + r (common.hpp, nb_kernels.hip k_latent_fwd), row = row_offset + batch
    position."""
    rows = row_offset + np.arange(B)
    return (philox_normal(seed, step, rows, np.arange(K)),
            philox_normal(seed, step, rows, NU_LANE + np.arange(R, dtype=np.uint64)))


NU_LANE = 0x80000000
