#!/usr/bin/env python3
"""Generate tests/golden/golden.json with the CPU ORACLE (Python restatement of the reference).

For every case: inputs are regenerated from `seed` by tests/common.make_inputs (their sha256 is
stored to pin the generator), the proof is produced by oracle.protocol.prove on the synthetic
power-11 ptau (tau = keccak256("kgs-bench-tau") mod r), and checked with the oracle verifier
(restated optimal-ate pairing) before it is written. The reference itself (JS + ffjavascript) is
not runnable offline, so these vectors are oracle outputs: "parity pinned" by
KATs + pairing verification, not by reference-run outputs.

`--lookup` writes tests/golden/lookup.json instead: lookup-argument proofs (SURVEY.md §8f N4;
include/kgs.h KGS_LOOKUP) for the reference's commented-out "standard lookup" case
(test/lookup_kzg_grandsum.test.js:24-44, common.reference_standard_lookup) and for random table
lookups (common.make_lookup_inputs). The reference has no lookup prover, so these pin the GPU path
to the oracle's restatement only ("parity unpinned" against the reference).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import common  # noqa: E402
from oracle import protocol as P  # noqa: E402

CASES = []
seed = 1000
for kind in ("grandsum", "grandproduct"):
    for npols, selected in ((1, False), (3, False), (1, True), (3, True)):
        for nbits in (1, 2, 3, 5, 8, 11):
            CASES.append(dict(kind=kind, nbits=nbits, npols=npols, selected=selected, seed=seed))
            seed += 1


LOOKUP_CASES = [dict(kind="lookup", gen="reference_standard", nbits=2, npols=1, unselected=0, seed=3)]
seed = 2000
for npols, unselected in ((1, 0), (1, 1), (3, 0), (2, 1)):
    for nbits in (1, 3, 5, 8):
        LOOKUP_CASES.append(dict(kind="lookup", gen="random_table", nbits=nbits, npols=npols,
                                 unselected=min(unselected, (1 << nbits) - 1), seed=seed))
        seed += 1


LOOKUP_CASES += [dict(kind="lookup", gen="dup_table", nbits=3, npols=1, unselected=0, seed=2100),
                 dict(kind="lookup", gen="dup_table", nbits=5, npols=1, unselected=0, seed=2101),
                 dict(kind="lookup", gen="all_zero", nbits=3, npols=1, unselected=8, seed=2102),
                 dict(kind="lookup", gen="random_table", nbits=3, npols=12, unselected=2, seed=2103)]


def lookup_inputs(c):
    if c["gen"] == "reference_standard":
        return common.reference_standard_lookup(c["seed"], c["nbits"])
    if c["gen"] == "dup_table":
        return common.lookup_dup_table(c["seed"], c["nbits"])
    if c["gen"] == "all_zero":
        return common.lookup_all_zero(c["seed"], c["nbits"])
    return common.make_lookup_inputs(c["seed"], c["nbits"], c["npols"], c["unselected"])


def main_lookup():
    path = common.oracle_ptau(11)
    srs = P.SRS(path, common.tau())
    out = {"ptau": {"power": 11, "tau": str(common.tau()), "writer": "oracle.ptau.write_synthetic_ptau"},
           "cases": []}
    for c in LOOKUP_CASES:
        Fs, Ts, sF, sM = lookup_inputs(c)
        eF = [P.EvalBuffer(x) for x in Fs]
        eT = [P.EvalBuffer(x) for x in Ts]
        trace = {}
        proof = P.prove("lookup", srs, eF if c["npols"] > 1 else eF[0], eT if c["npols"] > 1 else eT[0],
                        P.EvalBuffer(sF), P.EvalBuffer(sM), trace=trace)
        use_pairing = c["nbits"] <= 2
        assert P.verify("lookup", srs.ptau, proof, c["nbits"], tau=None if use_pairing else common.tau()), c
        rec = dict(c)
        rec["inputs_sha256"] = common.inputs_digest(Fs, Ts, sF, sM)
        rec["challenges"] = {k: str(v) for k, v in trace["challenges"].items()}
        rec["proof"] = {sec: {k: v.hex() for k, v in proof[sec].items()} for sec in ("commitments", "evaluations")}
        out["cases"].append(rec)
        print(c, "ok")
    with open(os.path.join(HERE, "lookup.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)


def run_case(c, srs, pairing=False):
    Fs, Ts, sF, sT = common.make_inputs(c["seed"], c["nbits"], c["npols"], c["selected"])
    eF = [P.EvalBuffer(x) for x in Fs]
    eT = [P.EvalBuffer(x) for x in Ts]
    trace = {}
    proof = P.prove(c["kind"], srs, eF if c["npols"] > 1 else eF[0], eT if c["npols"] > 1 else eT[0],
                    P.EvalBuffer(sF) if sF else None, P.EvalBuffer(sT) if sT else None, trace=trace)
    return Fs, Ts, sF, sT, proof, trace


def main():
    path = common.oracle_ptau(11)
    srs = P.SRS(path, common.tau())
    out = {"ptau": {"power": 11, "tau": str(common.tau()), "writer": "oracle.ptau.write_synthetic_ptau"},
           "cases": []}
    for c in CASES:
        Fs, Ts, sF, sT, proof, trace = run_case(c, srs)
        use_pairing = c["nbits"] <= 2
        ok = P.verify(c["kind"], srs.ptau, proof, c["nbits"], tau=None if use_pairing else common.tau())
        assert ok, c
        rec = dict(c)
        rec["inputs_sha256"] = common.inputs_digest(Fs, Ts, sF, sT)
        rec["challenges"] = {k: str(v) for k, v in trace["challenges"].items()}
        rec["proof"] = {sec: {k: v.hex() for k, v in proof[sec].items()} for sec in ("commitments", "evaluations")}
        out["cases"].append(rec)
        print(c, "ok")
    with open(os.path.join(HERE, "golden.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    if "--lookup" in sys.argv[1:]:
        main_lookup()
    else:
        main()
