"""Extracts the known-answer cases of pkg/inclusion/paths_test.go:12-...
(Test_calculateSubTreeRootCoordinates: start, end, maxDepth, minDepth ->
expected (depth, position) coordinates) into tests/golden/subtree_coords.json
(run here, where /root/reference exists)."""
import json
import os
import re

SRC = "/root/reference/pkg/inclusion/paths_test.go"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    src = open(SRC).read()
    body = src[src.index("func Test_calculateSubTreeRootCoordinates"):]
    cases = []
    sep = r",[^\n]*\s*"     # a field's comma, an optional trailing comment, the line break
    pat = (r'name:\s*"([^"]*)"' + sep + r"start:\s*(\d+)" + sep + r"end:\s*(\d+)" + sep + r"maxDepth:\s*(\d+)" + sep +
           r"minDepth:\s*(\d+)" + sep + r"expected:\s*\[\]coord\{(.*?)\n\t\t\t\},")
    for m in re.finditer(pat, body, re.S):
        coords = [[int(d), int(p)] for d, p in re.findall(r"depth:\s*(\d+),\s*position:\s*(\d+)", m.group(6))]
        cases.append({"name": m.group(1), "start": int(m.group(2)), "end": int(m.group(3)),
                      "max_depth": int(m.group(4)), "min_depth": int(m.group(5)), "expected": coords})
    with open(os.path.join(HERE, "subtree_coords.json"), "w") as f:
        json.dump({"source": "pkg/inclusion/paths_test.go (Test_calculateSubTreeRootCoordinates)", "cases": cases},
                  f, indent=1)
        f.write("\n")
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
