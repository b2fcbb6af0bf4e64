"""Numpy restatement of the device RNG streams (include/f16env.h) for tests: Philox4x32-10
(Salmon et al., SC'11; Random123 constants), the cfg5 random-IC box draw and the gust
Box-Muller normals. Vectorised over envs; independent of both the oracle and the kernel."""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32(key0, key1, c0, c1, c2, c3):
    """Arrays (broadcast) of uint32 -> (4, ...) uint32 outputs."""
    k0, k1 = np.asarray(key0, np.uint32), np.asarray(key1, np.uint32)
    c = [np.asarray(x, np.uint32) for x in np.broadcast_arrays(c0, c1, c2, c3)]
    k0, k1 = np.broadcast_to(k0, c[0].shape).copy(), np.broadcast_to(k1, c[0].shape).copy()
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c[0].astype(np.uint64)
            p1 = M1 * c[2].astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK).astype(np.uint32)
            c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
            k0 = k0 + W0
            k1 = k1 + W1
    return np.stack(c)


def random_ic(seed, gid, ep, lo, hi):
    """F16_FLAG_RANDOM_IC draw for envs gid (array), episode ep: (N, F16_IC_N) float64."""
    gid = np.asarray(gid, np.uint64)
    n_ic = len(lo)
    out = np.zeros((gid.size, n_ic))
    s0, s1 = np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF)
    for blk in range((n_ic + 3) // 4):
        o = philox4x32(s0, s1, (gid & MASK).astype(np.uint32), (gid >> np.uint64(32)).astype(np.uint32),
                       np.uint32(ep), np.uint32(0x52494300 + blk))
        for w in range(4):
            j = 4 * blk + w
            if j < n_ic:
                u = (o[w].astype(np.float64) + 0.5) * (1.0 / 4294967296.0)
                out[:, j] = lo[j] + (hi[j] - lo[j]) * u
    return out


def gust_normals(seed, gid, ep, step):
    """Three Box-Muller normals per env (float64), Philox (seed; gid, gid_hi ^ 'GUST', ep, step)."""
    gid = np.asarray(gid, np.uint64)
    s0, s1 = np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF)
    o = philox4x32(s0, s1, (gid & MASK).astype(np.uint32),
                   (gid >> np.uint64(32)).astype(np.uint32) ^ np.uint32(0x47555354),
                   np.asarray(ep, np.uint32), np.asarray(step, np.uint32))
    s24 = 1.0 / 16777216.0
    u1 = ((o[0] >> 8).astype(np.float64) + 0.5) * s24
    u2 = (o[1] >> 8).astype(np.float64) * s24
    u3 = ((o[2] >> 8).astype(np.float64) + 0.5) * s24
    u4 = (o[3] >> 8).astype(np.float64) * s24
    r1, r2 = np.sqrt(-2.0 * np.log(u1)), np.sqrt(-2.0 * np.log(u3))
    return np.stack([r1 * np.cos(2 * np.pi * u2), r1 * np.sin(2 * np.pi * u2), r2 * np.cos(2 * np.pi * u4)], -1)
