"""Extracts the known-answer cases of pkg/inclusion/paths_test.go into
tests/golden/ (run here, where /root/reference exists):
  - Test_calculateSubTreeRootCoordinates (:12-319): start, end, maxDepth,
    minDepth -> expected (depth, position) coordinates -> subtree_coords.json;
  - Test_genSubTreeRootPath (:321-339): depth, pos -> walk, and
    Test_calculateCommitPaths (:341-449): squareSize, start, blobLen ->
    expected paths at expected indexes (blobLen may name
    appconsts.DefaultSubtreeRootThreshold = v1.SubtreeRootThreshold = 64,
    pkg/appconsts/versioned_consts.go:30, pkg/appconsts/v1/app_consts.go:6)
    -> commit_paths.json."""
import json
import os
import re

SRC = "/root/reference/pkg/inclusion/paths_test.go"
HERE = os.path.dirname(os.path.abspath(__file__))
THRESHOLD = 64


def _walk(text):
    return [w == "WalkRight" for w in re.findall(r"Walk(?:Left|Right)", text)]


def _int(expr):
    expr = expr.replace("appconsts.DefaultSubtreeRootThreshold", str(THRESHOLD))
    if not re.fullmatch(r"[\d\s+*-]+", expr):
        raise ValueError(f"unexpected expression {expr!r}")
    return int(eval(expr))   # digits and + - * only (checked above)


def coordinate_cases(src):
    body = src[src.index("func Test_calculateSubTreeRootCoordinates"):src.index("func Test_genSubTreeRootPath")]
    cases = []
    sep = r",[^\n]*\s*"     # a field's comma, an optional trailing comment, the line break
    pat = (r'name:\s*"([^"]*)"' + sep + r"start:\s*(\d+)" + sep + r"end:\s*(\d+)" + sep + r"maxDepth:\s*(\d+)" + sep +
           r"minDepth:\s*(\d+)" + sep + r"expected:\s*\[\]coord\{(.*?)\n\t\t\t\},")
    for m in re.finditer(pat, body, re.S):
        coords = [[int(d), int(p)] for d, p in re.findall(r"depth:\s*(\d+),\s*position:\s*(\d+)", m.group(6))]
        cases.append({"name": m.group(1), "start": int(m.group(2)), "end": int(m.group(3)),
                      "max_depth": int(m.group(4)), "min_depth": int(m.group(5)), "expected": coords})
    return cases


def gen_path_cases(src):
    body = src[src.index("func Test_genSubTreeRootPath"):src.index("func Test_calculateCommitPaths")]
    return [{"depth": int(d), "pos": int(p), "expected": _walk(w)}
            for d, p, w in re.findall(r"\{(\d+),\s*(\d+),\s*\[\]WalkInstruction\{([^}]*)\}\}", body)]


def commit_path_cases(src):
    body = src[src.index("func Test_calculateCommitPaths"):src.index("func pathToString")]
    cases = []
    pat = (r'\{\s*"([^"]+)",\s*(\d+),\s*(\d+),\s*([^,\n]+),\s*\[\]path\{(.*?)\n\t\t\t\},\s*'
           r"\[\]int\{([\d,\s]*)\},\s*\},")
    for m in re.finditer(pat, body, re.S):
        paths = [{"row": int(r), "walk": _walk(w)}
                 for r, w in re.findall(r"row:\s*(\d+),\s*instructions:\s*\[\]WalkInstruction\{([^}]*)\}", m.group(5))]
        idx = [int(x) for x in re.findall(r"\d+", m.group(6))]
        cases.append({"name": m.group(1), "square_size": int(m.group(2)), "start": int(m.group(3)),
                      "blob_len": _int(m.group(4)), "expected_paths": paths, "expected_indexes": idx})
    return cases


def main():
    src = open(SRC).read()
    coords = coordinate_cases(src)
    with open(os.path.join(HERE, "subtree_coords.json"), "w") as f:
        json.dump({"source": "pkg/inclusion/paths_test.go (Test_calculateSubTreeRootCoordinates)", "cases": coords},
                  f, indent=1)
        f.write("\n")
    gen, commit = gen_path_cases(src), commit_path_cases(src)
    with open(os.path.join(HERE, "commit_paths.json"), "w") as f:
        json.dump({"source": "pkg/inclusion/paths_test.go (Test_genSubTreeRootPath, Test_calculateCommitPaths)",
                   "subtree_root_threshold": THRESHOLD, "gen_path": gen, "commit_paths": commit}, f, indent=1)
        f.write("\n")
    print(len(coords), "coordinate cases,", len(gen), "walk cases,", len(commit), "commit-path cases")


if __name__ == "__main__":
    main()
