#!/usr/bin/env python3
"""Compare dplasma_amd.models.qrtree against the reference oracle (tools/qrtree_oracle/oracle) and
(--write) store the digests of the oracle's trees as the parity fixture tests/fixtures/qrtree_ref.json.

Canonical form of a tree (both sides): per panel k, the GEQRT rows (getm order) and, per row m >= k,
[m, gettype, currpiv (-1 for m = k), nextpiv chain from mt, prevpiv chain from m]."""
from __future__ import annotations

import argparse
import hashlib
import itertools
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
ORACLE = os.path.join(ROOT, "tools", "qrtree_oracle", "oracle")
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "qrtree_ref.json")


def canon(t, mt, nt):
    steps = []
    for k in range(min(mt, nt)):
        rows = []
        for m in range(k, mt):
            nxt, n, g = [], t.nextpiv(k, m, mt), 0
            while n != mt and g < 4 * mt:
                nxt.append(n)
                n, g = t.nextpiv(k, m, n), g + 1
            prv, n, g = [], t.prevpiv(k, m, m), 0
            while n != mt and g < 4 * mt:
                prv.append(n)
                n, g = t.prevpiv(k, m, n), g + 1
            rows.append([m, t.gettype(k, m), t.currpiv(k, m) if m > k else -1, nxt, prv])
        steps.append({"k": k, "getm": [t.getm(k, i) for i in range(t.getnbgeqrf(k))], "rows": rows})
    return {"mt": mt, "nt": nt, "steps": steps}


def digest(obj) -> str:
    return hashlib.sha1(json.dumps(obj, separators=(",", ":"), sort_keys=True).encode()).hexdigest()[:16]


def configs(full=False):
    Ms = [1, 3, 4, 10, 17, 25] + ([40] if full else [])
    Ns = [1, 2, 5, 13]
    for llvl, a, m, n in itertools.product([0, 1, 2, 3, 4], [1, 2, 4], Ms, Ns):
        for tsrr in ([0, 1] if a > 1 else [0]):
            yield ("hqr", m, n, llvl, 0, a, 1, 0, tsrr)
            for dom, hlvl, p in itertools.product([0, 1], [0, 1, 2, 3, 4], [3, 5]):
                yield ("hqr", m, n, llvl, hlvl, a, p, dom, tsrr)
    for hlvl, p, cores, ratio, m, n in itertools.product([0, 1, 2, 3, 4], [1, 2, 3], [1, 2, 4], [1, 2], Ms, Ns):
        yield ("svd", m, n, hlvl, p, cores, ratio)
    for p, q, m, n in itertools.product([1, 4, 9], [2, 4, 9], Ms, Ns):
        yield ("sys", m, n, p, q)


def ours(cfg):
    from dplasma_amd.models import qrtree as Q
    kind, m, n = cfg[0], cfg[1], cfg[2]
    if kind == "hqr":
        llvl, hlvl, a, p, dom, tsrr = cfg[3:]
        t = Q.HQRTree(m, n, llvl, hlvl, a, p, dom, tsrr)
    elif kind == "svd":
        hlvl, p, cores, ratio = cfg[3:]
        t = Q.SVDTree(m, n, hlvl, p, cores, ratio)
    else:
        p, q = cfg[3:]
        t = Q.SystolicTree(m, n, p, q)
    return canon(t, m, n)


def oracle(cfg):
    r = subprocess.run([ORACLE, cfg[0], *map(str, cfg[1:])], capture_output=True, text=True, timeout=60)
    if r.returncode != 0:
        return None
    return json.loads(r.stdout)


def key(cfg):
    return " ".join(map(str, cfg))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--write", action="store_true", help="(re)write the fixture from the oracle")
    ap.add_argument("--kind", default=None)
    ap.add_argument("--show", type=int, default=3, help="print the first N mismatching configs")
    args = ap.parse_args()
    cfgs = [c for c in configs() if args.kind is None or c[0] == args.kind]
    if args.write:
        ref = {}
        for c in cfgs:
            o = oracle(c)
            if o is not None:
                ref[key(c)] = digest(o)
        os.makedirs(os.path.dirname(FIXTURE), exist_ok=True)
        json.dump({"source": "tools/qrtree_oracle/oracle built from the reference's dplasma_hqr.c / "
                             "dplasma_systolic_qr.c; sha1[:16] of the canonical tree (compare.py canon)",
                   "trees": ref}, open(FIXTURE, "w"), indent=0, sort_keys=True)
        print(f"wrote {len(ref)} digests to {FIXTURE}")
        return
    ref = json.load(open(FIXTURE))["trees"]
    bad = {}
    shown = 0
    for c in cfgs:
        k = key(c)
        if k not in ref:
            continue
        try:
            d = digest(ours(c))
        except Exception as e:  # noqa: BLE001
            d = f"error {e}"
        if d != ref[k]:
            tag = c[0] if c[0] != "hqr" else f"hqr l{c[3]} h{c[4]} dom{c[7]} rr{c[8]} p{'>1' if c[6] > 1 else '1'}"
            bad.setdefault(tag, []).append(k)
            if shown < args.show and os.path.exists(ORACLE):
                shown += 1
                print("MISMATCH", k)
    tot = len([c for c in cfgs if key(c) in ref])
    nbad = sum(len(v) for v in bad.values())
    print(f"{tot - nbad}/{tot} trees identical to the reference")
    for tag, v in sorted(bad.items()):
        print(f"  {len(v):5d}  {tag}")


if __name__ == "__main__":
    main()
