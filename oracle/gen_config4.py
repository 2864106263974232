"""Config-4 fixture: oracle digests of the 128 distinct k=128 squares one GPU
of an 8-GPU node processes (BASELINE.json configs[3]: 1024 squares, seeds
0..1023, rank g takes [128g, 128g+128)).

TEST INFRASTRUCTURE.  `python oracle/gen_config4.py` writes
tests/golden/config4_k128.json: per square index the SHA-256 of its ODS, EDS,
row roots, column roots and its data root, from the C oracle
(oracle/cda_oracle.c, the CPU restatement pinned by the reference's golden
vectors and mainnet block 408).  `--k 512 --count 2 --out
tests/golden/k512.json` writes the same for config 3's squares 0 and 1.
`--first 128 --count 896 --roots-only --out tests/golden/config4_k128_rest.json`
writes the data root and root digests of the other seven ranks' squares
(every rank's shard is then checked, not only rank 0's).
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "celestia-app_amd"))
import coracle  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(HERE), "tests", "golden")


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--count", type=int, default=128)
    ap.add_argument("--out", default=os.path.join(GOLDEN, "config4_k128.json"))
    ap.add_argument("--roots-only", action="store_true", help="data root and root digests only (smaller fixture)")
    a = ap.parse_args()
    first, count, k = a.first, a.count, a.k
    from celestia_da import testfactory   # the bench's generator must agree with the oracle's
    out = {"k": k, "first": first, "count": count,
           "generator": "testfactory mirror, SplitMix64 seed 0xCE1E57A0 + square index (SURVEY.md 8(d))",
           "squares": {}}
    for i in range(first, first + count):
        ods = coracle.random_square(k, i)
        if i % 32 == 0 or k > 128:
            assert np.array_equal(ods, testfactory.random_square(k, i))
        eds, rows, cols, root = coracle.cpu_baseline(ods, os.cpu_count() or 8)
        rec = {"row_roots_sha256": digest(rows), "col_roots_sha256": digest(cols), "data_root": root.hex()}
        if not a.roots_only:
            rec.update(ods_sha256=digest(ods), eds_sha256=digest(eds))
        out["squares"][str(i)] = rec
    with open(a.out, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
