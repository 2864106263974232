"""Generate tests/golden fixtures from the reference's own data and the oracle.

TEST INFRASTRUCTURE.  Run in the container that has /root/reference:
    python oracle/gen_golden.py
Outputs (committed; the GPU box never reads /root/reference):
  tests/golden/block408_ods.bin.gz  -- ODS of mainnet block 408 (k=32) built by
      oracle/square.py from x/blob/test/testdata/block_response.json
  tests/golden/block408_txs.json.gz -- the block's txs (base64), square size
      and header.data_hash, copied from that reference fixture (data only) so
      GPU tests can run square construction without /root/reference
  tests/golden/golden.json          -- expected data roots: the reference's
      golden hashes (pkg/da/data_availability_header_test.go) and the block's
      data_hash, plus oracle digests of random squares (seeded SplitMix64).
"""
import base64
import gzip
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import coracle  # noqa: E402
import pyref  # noqa: E402
import square  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    os.makedirs(OUT, exist_ok=True)
    g = {"reference_golden": {
        # pkg/da/data_availability_header_test.go:17-24, :29, :45, :51
        "nil_dah": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
        "min_dah_k1": "3d96b7d238e7e0456f6af8e7cdf0a67bd6cf9c2089ecb559c659dcaa1f880353",
        "constant_k2": "b56e4d251ac266f4b91cc5464b3fc7efcbdc888064647496d13133f0dc65ac25",
        "constant_k128": "0bd3abeeacfbb0b92dfbdac4a154868e3c4e79666f7fcf6c620bb90dd3a0dcf0",
    }}
    txs, k, data_hash = square.load_block(os.path.join(REF, "x/blob/test/testdata/block_response.json"))
    with gzip.open(os.path.join(OUT, "block408_txs.json.gz"), "wt", compresslevel=9) as f:
        json.dump({"height": 408, "square_size": k, "data_hash": data_hash.hex(),
                   "txs": [base64.b64encode(t).decode() for t in txs]}, f)
    ods = np.frombuffer(b"".join(square.construct(txs, k)), dtype=np.uint8).reshape(k * k, 512)
    with gzip.open(os.path.join(OUT, "block408_ods.bin.gz"), "wb", compresslevel=9) as f:
        f.write(ods.tobytes())
    eds, rows, cols, root = coracle.extend_dah(ods)
    assert root == data_hash, "oracle does not reproduce block 408 data_hash"
    g["block408"] = {"k": k, "data_hash": data_hash.hex(), "ods_sha256": digest(ods), "eds_sha256": digest(eds),
                     "row_roots_sha256": digest(rows), "col_roots_sha256": digest(cols),
                     "source": "x/blob/test/testdata/block_response.json (height 408, header.data_hash)"}
    rnd = {}
    for k in (1, 2, 4, 8, 16, 32, 64, 128):
        ods = coracle.random_square(k, 7)
        eds, rows, cols, root = coracle.extend_dah(ods) if k < 64 else coracle.cpu_baseline(ods, 8)
        if k <= 8:
            e2, r2, c2, root2 = pyref.extend_and_dah(pyref.ods_from_shares(pyref.random_namespaced_square(k, 7)))
            assert root2 == root
        rnd[str(k)] = {"seed_index": 7, "ods_sha256": digest(ods), "eds_sha256": digest(eds),
                       "row_roots_sha256": digest(rows), "col_roots_sha256": digest(cols), "data_root": root.hex()}
    g["random_squares"] = rnd
    with open(os.path.join(OUT, "golden.json"), "w") as f:
        json.dump(g, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
