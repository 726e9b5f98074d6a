"""Test-matrix generators: pltmg (LAWN 263 gallery) and latms.

Reference: ``src/zpltmg_wrapper.c`` (dispatch :480-548), ``src/cores/core_zpltmg.c``
(element formulas), ``core_zpltmg_{chebvand,circul,condex,fiedler,hankel,toeppd}.c``,
``src/zlatms_wrapper.c`` (D(i) = 1 - i/(N-1) (1 - 1/cond), then random unitary
factors from geqrf/unmqr).  Type codes: ``src/include/dplasma/constants.h:163-207``.

Every generator is a function of the GLOBAL element indices (and of the 64-bit
LCG stream for the random-vector based ones), so the result is identical for
any tiling or process grid -- the property the reference gets from
``Rnd64_jump`` (``src/cores/random.h:20-41``).  Formulas are evaluated on the
matrix's own device, one local tile column at a time (all its local tiles
stacked); the random base of Demmel / Langou comes from the GPU LCG generator
(plrnt) and the O(N) random vectors of the vector-based types are generated once
and moved to the device -- nothing is assembled on the host.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..constants import dplasmaConjTrans, dplasmaLeft, dplasmaNoTrans, dplasmaRight, dplasmaUpperLower
from ..utils import lcg

(dplasmaMatrixRandom, dplasmaMatrixHadamard, dplasmaMatrixHouse, dplasmaMatrixParter, dplasmaMatrixRis,
 dplasmaMatrixKms, dplasmaMatrixToeppen, dplasmaMatrixCondex, dplasmaMatrixMoler, dplasmaMatrixCircul,
 dplasmaMatrixRandcorr, dplasmaMatrixPoisson, dplasmaMatrixHankel, dplasmaMatrixJordbloc, dplasmaMatrixCompan,
 dplasmaMatrixPei, dplasmaMatrixRandcolu, dplasmaMatrixSprandn, dplasmaMatrixRiemann, dplasmaMatrixCompar,
 dplasmaMatrixTridiag, dplasmaMatrixChebspec, dplasmaMatrixLehmer, dplasmaMatrixToeppd, dplasmaMatrixMinij,
 dplasmaMatrixRandsvd, dplasmaMatrixForsythe, dplasmaMatrixFiedler, dplasmaMatrixDorr, dplasmaMatrixDemmel,
 dplasmaMatrixChebvand, dplasmaMatrixInvhess, dplasmaMatrixProlate, dplasmaMatrixFrank, dplasmaMatrixCauchy,
 dplasmaMatrixHilb, dplasmaMatrixLotkin, dplasmaMatrixKahan, dplasmaMatrixOrthog, dplasmaMatrixWilkinson,
 dplasmaMatrixFoster, dplasmaMatrixWright, dplasmaMatrixLangou) = range(43)

UNAVAILABLE = {dplasmaMatrixToeppen, dplasmaMatrixRandcorr, dplasmaMatrixPoisson, dplasmaMatrixJordbloc,
               dplasmaMatrixPei, dplasmaMatrixRandcolu, dplasmaMatrixSprandn, dplasmaMatrixCompar,
               dplasmaMatrixTridiag, dplasmaMatrixChebspec, dplasmaMatrixRandsvd, dplasmaMatrixForsythe,
               dplasmaMatrixProlate, dplasmaMatrixFrank, dplasmaMatrixKahan}


def _rand_block(dtype, gM, i0, j0, rows, cols, seed):
    """plrnt values of the global block (i0:i0+rows, j0:j0+cols) of a gM-row matrix (host, float64/complex128)."""
    return torch.from_numpy(np.ascontiguousarray(lcg.rnd_block(i0, j0, rows, cols, gM, seed, dtype.is_complex)))


def _rand_vec(dtype, n, seed, row=False):
    """Random vector = the first column (or row) of a plrnt matrix."""
    if row:
        return _rand_block(dtype, 1, 0, 0, 1, n, seed)[0]
    return _rand_block(dtype, n, 0, 0, n, 1, seed)[:, 0]


def _formula(t, dtype, gM, gN, I, J, seed, cache):
    """Element values at global 0-based index grids I, J (host tensors)."""
    cd = torch.complex128 if dtype.is_complex else torch.float64
    If, Jf = I.to(torch.float64), J.to(torch.float64)
    Ii, Ji = I + 1, J + 1  # 1-based
    if t == dplasmaMatrixHadamard:
        x = torch.bitwise_and(I, J)
        pc = torch.zeros_like(x)
        while bool((x > 0).any()):
            pc += x & 1
            x = x >> 1
        return (1.0 - 2.0 * (pc % 2).to(torch.float64)).to(cd)
    if t == dplasmaMatrixParter:
        return (1.0 / (If - Jf + 0.5)).to(cd)
    if t == dplasmaMatrixRis:
        return (0.5 / (gM - If - Jf - 0.5)).to(cd)
    if t == dplasmaMatrixKms:
        return torch.pow(torch.tensor(0.5, dtype=torch.float64), (If - Jf).abs()).to(cd)
    if t == dplasmaMatrixMoler:
        return torch.where(I == J, If + 1.0, torch.minimum(If, Jf) - 1.0).to(cd)
    if t == dplasmaMatrixRiemann:
        ii, jj = I + 2, J + 2
        return torch.where(jj % ii == 0, (ii - 1).to(torch.float64), torch.full_like(If, -1.0)).to(cd)
    if t == dplasmaMatrixLehmer:
        return torch.where(Jf >= If, (Ii.double() / Ji.double()), (Ji.double() / Ii.double())).to(cd)
    if t == dplasmaMatrixMinij:
        return torch.minimum(Ii, Ji).to(cd)
    if t == dplasmaMatrixInvhess:
        return torch.where(Ji <= Ii, Ji.double(), -Ii.double()).to(cd)
    if t == dplasmaMatrixCauchy:
        return (1.0 / (Ii + Ji).double()).to(cd)
    if t == dplasmaMatrixHilb:
        return (1.0 / (If + Jf + 1.0)).to(cd)
    if t == dplasmaMatrixLotkin:
        return torch.where(I == 0, torch.ones_like(If), 1.0 / (If + Jf + 1.0)).to(cd)
    if t == dplasmaMatrixOrthog:
        scale = math.pi / (gN + 1.0)
        return (math.sqrt(2.0 / (gN + 1.0)) * torch.sin(Ii.double() * Ji.double() * scale)).to(cd)
    if t == dplasmaMatrixWilkinson:
        dist = torch.minimum(gN - 1 - I, I).double()
        v = torch.where(I == J, (gN - 2.0 * dist - 1.0) / 2.0,
                        torch.where((I - J).abs() == 1, torch.ones_like(If), torch.zeros_like(If)))
        return v.to(cd)
    if t == dplasmaMatrixFoster:
        k = h = c = 1.0
        diag = torch.where(J == 0, torch.ones_like(If),
                           torch.where(J == gN - 1, torch.full_like(If, 1 - 1 / c - k * h / 2),
                                       torch.full_like(If, 1 - k * h / 2)))
        off = torch.where(J == 0, torch.full_like(If, -k * h / 2),
                          torch.where(J == gN - 1, torch.full_like(If, -1 / c),
                                      torch.where(I > J, torch.full_like(If, -k * h), torch.zeros_like(If))))
        return torch.where(I == J, diag, off).to(cd)
    if t == dplasmaMatrixWright:
        v = torch.zeros_like(If)
        v = torch.where(I == J, torch.ones_like(If), v)
        even, odd = (J % 2 == 0), (J % 2 == 1)
        v = torch.where((I == J + 2) & even, torch.full_like(If, -0.9048), v)
        v = torch.where((I == J + 3) & even, torch.full_like(If, -1.2092), v)
        v = torch.where((I == J + 2) & odd, torch.full_like(If, -0.8270), v)
        v = torch.where((I == J + 3) & odd, torch.full_like(If, -1.3499), v)
        v = torch.where((J == gM - 2) & (I == 0), torch.ones_like(If), v)
        v = torch.where((J == gM - 1) & (I == 1), torch.ones_like(If), v)
        return v.to(cd)
    if t == dplasmaMatrixDorr:
        theta, h = 0.01, 1.0 / (gN + 1.0)
        term = theta / (h * h)
        half = (gN + 1) // 2
        c = J
        lo = c < half
        diag = torch.where(lo, 2 * term + (0.5 - (Jf + 1) * h) / h, 2 * term - (0.5 - (Jf + 1) * h) / h)
        sup = torch.where(lo, -term - (0.5 - Jf * h) / h,
                          torch.where(c == half, -term - (0.5 - Jf * h) / h, torch.full_like(Jf, -term)))
        sub = torch.where(lo, torch.where(c + 1 == half, -term + (0.5 - (Jf + 2) * h) / h,
                                          torch.full_like(Jf, -term)),
                          -term + (0.5 - (Jf + 2) * h) / h)
        v = torch.where(I == J, diag, torch.where(I == J - 1, sup, torch.where(I == J + 1, sub,
                                                                                 torch.zeros_like(If))))
        return v.to(cd)
    dev = I.device
    if t == dplasmaMatrixCompan:
        if "compan" not in cache:
            r = _rand_vec(dtype, gN, seed, row=True)
            v0 = _rand_block(dtype, 1, 0, 0, 1, 1, seed)[0, 0]
            cache["compan"] = (r / v0).to(dev)
        r = cache["compan"]
        v = torch.where(I == J + 1, torch.ones_like(If), torch.zeros_like(If)).to(cd)
        first = r[J.clamp(max=gN - 1)]
        first = torch.where(J == 0, torch.zeros_like(first), first)
        return torch.where(I == 0, first, v)
    if t == dplasmaMatrixDemmel:
        base = cache["rand"](I, J)
        d = torch.pow(torch.tensor(10.0, dtype=torch.float64), 14.0 * If / gM)
        return base * (d * torch.where(I == J, torch.ones_like(If), torch.full_like(If, 1e-7))).to(cd)
    if t == dplasmaMatrixLangou:
        base = cache["rand"](I, J)
        eps = float(torch.finfo(torch.float64 if dtype in (torch.float64, torch.complex128) else torch.float32).eps)
        mn = min(gM, gN)
        sel = (J >= mn // 4) & (J < mn // 2) & (I >= J)
        return torch.where(sel, base * eps, base)
    if t == dplasmaMatrixCircul:
        if "vec" not in cache:
            cache["vec"] = _rand_vec(dtype, gN, seed).to(dev)
        return cache["vec"][(J - I) % gN]
    if t == dplasmaMatrixFiedler:
        if "vec" not in cache:
            cache["vec"] = _rand_vec(dtype, max(gM, gN), seed).to(dev)
        v = cache["vec"]
        return (v[I] - v[J]).abs().to(cd)
    if t == dplasmaMatrixHankel:
        if "vec" not in cache:
            cache["vec"] = _rand_vec(dtype, gM + gN, seed).to(dev)
        return cache["vec"][I + J]
    if t == dplasmaMatrixChebvand:
        step = 1.0 / (gN - 1.0) if gN > 1 else 0.0
        p = Jf * step
        maxi = int(I.max()) + 1 if I.numel() else 1
        T0, T1 = torch.ones_like(p), p.clone()
        out = torch.zeros_like(p)
        out = torch.where(I == 0, T0, out)
        out = torch.where(I == 1, T1, out)
        for k in range(2, maxi):
            T0, T1 = T1, 2 * p * T1 - T0
            out = torch.where(I == k, T1, out)
        return out.to(cd)
    if t == dplasmaMatrixToeppd:
        if "toeppd" not in cache:
            # A(i, j) = t(i - j) = sum_k w_k cos(theta_k (i - j)): the 2N - 1 values once, in chunks
            W = _rand_block(dtype, 2, 0, 0, 2, gM, seed).real.to(dev)
            w, th = W[0] + 0.5, 2 * math.pi * (W[1] + 0.5)
            n = max(gM, gN)
            d = torch.arange(-(n - 1), n, dtype=torch.float64, device=dev)
            tv = torch.empty_like(d)
            step = max(1, (1 << 24) // max(1, gM))
            for a in range(0, len(d), step):
                tv[a:a + step] = (w.view(1, -1) * torch.cos(th.view(1, -1) * d[a:a + step].view(-1, 1))).sum(1)
            cache["toeppd"] = (tv, n - 1)
        tv, z = cache["toeppd"]
        return tv[(I - J) + z].to(cd)
    if t == dplasmaMatrixHouse:
        if "vec" not in cache:
            cache["vec"] = _rand_vec(dtype, gM, seed).to(dev)
        v = cache["vec"]
        tau = 2.0 / float((v.abs() ** 2).sum())
        return torch.where(I == J, torch.ones_like(If), torch.zeros_like(If)).to(cd) - tau * v[I] * v[J].conj()
    if t == dplasmaMatrixCondex:
        if "condex" not in cache:
            n = gM
            X = torch.zeros(n, 3, dtype=cd)
            X[:, 0] = 1.0
            X[0, 1] = 1.0
            i = torch.arange(n, dtype=torch.float64)
            X[:, 2] = ((-1.0) ** i) * (1.0 + i / max(gN - 1, 1))
            Q, _ = torch.linalg.qr(X)
            cache["condex"] = Q.to(dev)
        Q = cache["condex"]
        theta = 100.0
        return torch.where(I == J, torch.full_like(If, 1.0 + theta), torch.zeros_like(If)).to(cd) - \
            theta * (Q[I] * Q[J].conj()).sum(-1)
    raise ValueError(f"unsupported matrix type {t}")


def pltmg(ctx, mtxtype: int, A, seed: int = 3872):
    """Generate a LAWN-263 test matrix into A (dplasma_zpltmg); returns 0, or -2 for unavailable types."""
    if mtxtype in UNAVAILABLE or not (0 <= mtxtype <= 42):
        return -2
    from .aux import plrnt
    if mtxtype == dplasmaMatrixRandom:
        plrnt(ctx, A, seed)
        return 0
    if mtxtype in (dplasmaMatrixHadamard,) and (A.m != A.n or A.m & (A.m - 1)):
        return -2
    gM, gN = A.m, A.n
    cache = {}
    dev = A.device
    if mtxtype in (dplasmaMatrixDemmel, dplasmaMatrixLangou):
        plrnt(ctx, A, seed)          # the random base, by the GPU LCG generator, transformed in place

    def rand(I, J):
        return cache["base"]
    cache["rand"] = rand
    bycol = {}
    for (m, n) in A.local_tiles():
        bycol.setdefault(n, []).append(m)
    for n, ms in sorted(bycol.items()):
        # every local tile of tile column n at once: rows stacked, one formula evaluation
        c0, cols = n * A.nb, A.tile_cols(n)
        rows = torch.cat([torch.arange(m * A.mb, m * A.mb + A.tile_rows(m), device=dev) for m in ms])
        I = rows.view(-1, 1).expand(len(rows), cols)
        J = torch.arange(c0, c0 + cols, device=dev).view(1, -1).expand(len(rows), cols)
        if "rand" in cache and mtxtype in (dplasmaMatrixDemmel, dplasmaMatrixLangou):
            cache["base"] = torch.cat([A.tile(m, n) for m in ms]).to(torch.complex128 if A.dtype.is_complex
                                                                      else torch.float64)
        vals = _formula(mtxtype, A.dtype, gM, gN, I, J, seed, cache)
        if not A.dtype.is_complex and vals.is_complex():
            vals = vals.real
        vals = vals.to(A.dtype)
        r = 0
        for m in ms:
            h = A.tile_rows(m)
            A.tile(m, n).copy_(vals[r:r + h])
            r += h
    if ctx.is_gpu:
        torch.cuda.synchronize(A.device)
    return 0


def latms(ctx, mtxtype, cond: float, A, seed: int = 3872):
    """Random matrix with prescribed singular values D(i) = 1 - i/(N-1)(1 - 1/cond) (dplasma_zlatms).

    mtxtype General: A = Q1 D Q2 with random unitary factors (geqrf of plrnt
    matrices); Hermitian/symmetric: A = Q D Q^H."""
    from . import qr
    from ..constants import dplasmaGeneral
    n = A.n
    tmp = 1.0 / cond
    alp = (1.0 - tmp) / (n - 1) if n > 1 else 0.0
    for (m, nn) in A.local_tiles():
        t = A.tile(m, nn)
        t.zero_()
        if m == nn:
            k = min(A.tile_rows(m), A.tile_cols(nn))
            g = torch.arange(k, dtype=torch.float64) + nn * A.nb
            d = (n - g - 1) * alp + tmp
            d = torch.where(g == 0, torch.ones_like(d), d)
            t.diagonal()[:k].copy_(d.to(A.dtype).to(A.device))
    ib = 32 if A.nb >= 32 else A.nb

    def qfactor(rows, s):
        Qm = A.like(lm=rows, ln=rows, name="Q")
        from .aux import plrnt
        plrnt(ctx, Qm, s)
        T = Qm.like(lm=Qm.mt * ib, ln=Qm.n, name="T")
        T2 = T.__class__(A.dtype, ib, Qm.nb, Qm.mt * ib, Qm.n, P=Qm.grid.P, Q=Qm.grid.Q, rank=Qm.rank,
                         device=Qm.device)
        qr.geqrf(ctx, Qm, T2)
        return Qm, T2
    if mtxtype == dplasmaGeneral:
        Q1, T1 = qfactor(A.m, seed)
        qr.unmqr(ctx, dplasmaLeft, dplasmaNoTrans, Q1, T1, A)
        Q2, T2 = qfactor(A.n, seed + 1)
        qr.unmqr(ctx, dplasmaRight, dplasmaNoTrans, Q2, T2, A)
    else:
        Q1, T1 = qfactor(A.m, seed)
        qr.unmqr(ctx, dplasmaLeft, dplasmaNoTrans, Q1, T1, A)
        qr.unmqr(ctx, dplasmaRight, dplasmaConjTrans, Q1, T1, A)
    return 0
