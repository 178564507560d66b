"""Relational truth for the measured configs at full size, by aggregate push-down.  A checker
(test infrastructure): sums over join results computed from per-key counts, never materialising
the join -- exact mod 2^64.

chain:  R0.c1 = R1.c0, R1.c1 = R2.c0, R2.c1 = R3.c0 with an optional row filter on R3.
"""
import numpy as np

M64 = (1 << 64) - 1


def _bincount_u(keys, weights, domain):
    """exact integer bincount (weights are small non-negative ints; float64 is exact < 2^53)"""
    if weights is None:
        return np.bincount(keys.astype(np.int64), minlength=domain).astype(np.uint64)
    return np.rint(np.bincount(keys.astype(np.int64), weights=weights.astype(np.float64),
                               minlength=domain)).astype(np.uint64)


def chain4_sums(rels, domain, r3_mask=None):
    """(count of R3 rows passing the filter, chain rows, [sum R1.c2, sum R2.c2, sum R3.c2]) mod 2^64"""
    R0, R1, R2, R3 = rels
    m3 = np.ones(len(R3[0]), dtype=bool) if r3_mask is None else r3_mask
    cnt3 = _bincount_u(R3[0][m3], None, domain)                 # R3 rows per join key
    down2 = cnt3[R2[1]]                                          # (r3) continuations of each r2
    cnt2 = _bincount_u(R2[0], down2, domain)
    down1 = cnt2[R1[1]]
    up1 = _bincount_u(R0[1], None, domain)[R1[0]]                # r0 partners of each r1
    up2 = _bincount_u(R1[1], up1, domain)[R2[0]]
    up3 = _bincount_u(R2[1], up2, domain)[R3[0]]
    with np.errstate(over="ignore"):
        mult1 = up1 * down1
        mult2 = up2 * down2
        mult3 = np.where(m3, up3, np.uint64(0))
        s1 = np.sum(mult1 * R1[2], dtype=np.uint64)
        s2 = np.sum(mult2 * R2[2], dtype=np.uint64)
        s3 = np.sum(mult3 * R3[2], dtype=np.uint64)
    rows = int(np.sum(mult3, dtype=np.uint64))
    return int(m3.sum()), rows, [int(s1), int(s2), int(s3)]


def pair_sums(R0, R1, domain):
    """2-relation R0.c1 = R1.c0: (pairs, sum R0.c2, sum R1.c2)"""
    cs = _bincount_u(R1[0], None, domain)[R0[1]]
    cr = _bincount_u(R0[1], None, domain)[R1[0]]
    with np.errstate(over="ignore"):
        return int(np.sum(cs, dtype=np.uint64)), int(np.sum(cs * R0[2], dtype=np.uint64)), \
            int(np.sum(cr * R1[2], dtype=np.uint64))


def sharded_pair_sums(kR, vR, kS, vS, domain, shards):
    """R.key = S.key: (pairs, sum over pairs of vR, sum over pairs of vS) mod 2^64, per key range
    [lo, hi): counts cR, cS over the range, pairs += sum cR * cS, sums += cS[kR] * vR / cR[kS] * vS
    (int64 arithmetic wraps: exact mod 2^64)"""
    import torch
    pairs = sa = sb = 0
    for s in range(shards):
        lo, hi = domain * s // shards, domain * (s + 1) // shards
        mR = (kR >= lo) & (kR < hi)
        mS = (kS >= lo) & (kS < hi)
        r_idx, s_idx = kR[mR] - lo, kS[mS] - lo
        cR = torch.bincount(r_idx, minlength=hi - lo)
        cS = torch.bincount(s_idx, minlength=hi - lo)
        pairs += int((cR * cS).sum().item())
        sa += int((cS[r_idx] * vR[mR]).sum().item())
        sb += int((cR[s_idx] * vS[mS]).sum().item())
        del mR, mS, r_idx, s_idx, cR, cS
    return pairs & M64, sa & M64, sb & M64
