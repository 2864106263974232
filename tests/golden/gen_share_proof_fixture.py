"""Extracts the reference's valid ShareProof test vector into
tests/golden/share_proof_valid.json (run here, where /root/reference exists;
the GPU box reads only the JSON).

Source data (byte literals, not code): pkg/proof/share_proof_test.go:77-93
validShareProof() and pkg/proof/row_proof_test.go:68-89 (`root`,
validRowProof()) -- a one-share proof of a transaction share from
TestNewShareInclusionProof, k = 32 (64-leaf rows, 128 DAH roots).
"""
import json
import os
import re

REF = "/root/reference/pkg/proof"
HERE = os.path.dirname(os.path.abspath(__file__))
BYTES = re.compile(r"\{((?:0x[0-9a-f]+,\s*)*0x[0-9a-f]+)\}")


def byte_lists(text):
    return [bytes(int(x, 16) for x in m.split(",")) for m in BYTES.findall(text)]


def func_body(src, name):
    i = src.index(f"func {name}()")
    j = src.index("\n}\n", i)
    return src[i:j]


def field(body, name):
    m = re.search(rf"{name}:\s*(.*)", body)
    return m.group(1)


def main():
    sp_src = open(os.path.join(REF, "share_proof_test.go")).read()
    rp_src = open(os.path.join(REF, "row_proof_test.go")).read()
    sp = func_body(sp_src, "validShareProof")
    rp = func_body(rp_src, "validRowProof")
    root = byte_lists(re.search(r"var root = \[\]byte(\{[^}]*\})", rp_src).group(1))[0]
    data = byte_lists(field(sp, "Data"))
    nodes = byte_lists(field(sp, "Nodes"))
    ns_id = bytes(int(x) for x in re.search(r"NamespaceId:\s*\[\]byte\{([^}]*)\}", sp).group(1).split(","))
    out = {
        "source": "pkg/proof/share_proof_test.go:77-93, pkg/proof/row_proof_test.go:68-89",
        "root": root.hex(),
        "data": [d.hex() for d in data],
        "share_proofs": [{"start": int(re.search(r"Start:\s*(\d+)", sp).group(1)),
                          "end": int(re.search(r"End:\s*(\d+)", sp).group(1)),
                          "nodes": [n.hex() for n in nodes]}],
        "namespace_id": ns_id.hex(),
        "namespace_version": int(re.search(r"NamespaceVersion:\s*uint32\((\d+)\)", sp).group(1)),
        "row_proof": {
            "row_roots": [r.hex() for r in byte_lists(field(rp, "RowRoots"))],
            "proofs": [{"total": int(re.search(r"Total:\s*(\d+)", rp).group(1)),
                        "index": int(re.search(r"Index:\s*(\d+)", rp).group(1)),
                        "leaf_hash": byte_lists(field(rp, "LeafHash"))[0].hex(),
                        "aunts": [a.hex() for a in byte_lists(field(rp, "Aunts"))]}],
            "start_row": int(re.search(r"StartRow:\s*(\d+)", rp).group(1)),
            "end_row": int(re.search(r"EndRow:\s*(\d+)", rp).group(1)),
        },
    }
    with open(os.path.join(HERE, "share_proof_valid.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
