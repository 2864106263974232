"""Single-square latency (configs 2 and 3) of the latency-bound tails under
environment variants: each variant runs in its own process (the library reads
CDA_* knobs once).  Usage: python tools/tail_ab.py [k ...]
Prints per variant and k: median wall ms of extend_dah_device and the data
root (all variants must agree)."""
import json
import os
import subprocess
import sys

VARIANTS = {
    "pair+rfc (default)": {},
    "no pair": {"CDA_TOP_PAIR": "0"},
    "no rfc-in-top": {"CDA_TOP_RFC": "0"},
    "neither": {"CDA_TOP_PAIR": "0", "CDA_TOP_RFC": "0"},
}

CHILD = r'''
import os, sys, time, json
import numpy as np, torch
sys.path.insert(0, os.path.join(os.environ["GRAFT_ROOT"], "celestia-app_amd"))
from celestia_da import Context, testfactory
out = {}
ctx = Context(0)
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
for k in [int(x) for x in sys.argv[1:]]:
    W = 2 * k
    o = torch.from_numpy(testfactory.random_square(k, 0)).to(dev)
    e = torch.empty(W * W * 512, dtype=torch.uint8, device=dev)
    r = torch.empty(W * 90, dtype=torch.uint8, device=dev)
    c = torch.empty(W * 90, dtype=torch.uint8, device=dev)
    g = torch.empty(32, dtype=torch.uint8, device=dev)
    st = torch.empty(1, dtype=torch.int32, device=dev)
    lat = []
    for i in range(25):
        torch.cuda.synchronize(dev)
        a = time.perf_counter()
        ctx.extend_dah_device(o.data_ptr(), k, 1, e.data_ptr(), r.data_ptr(), c.data_ptr(), g.data_ptr(),
                              st.data_ptr(), s)
        torch.cuda.synchronize(dev)
        lat.append(time.perf_counter() - a)
    out[k] = {"ms": 1e3 * float(np.median(lat[5:])), "root": bytes(g.cpu().numpy()).hex()}
    del o, e
    torch.cuda.empty_cache()
print("RESULT " + json.dumps(out))
'''


def main():
    global VARIANTS
    if os.environ.get("TAIL_AB_VARIANTS"):   # JSON {name: {env}} replaces the default set
        VARIANTS = json.loads(os.environ["TAIL_AB_VARIANTS"])
    ks = sys.argv[1:] or ["128", "512"]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    rounds = int(os.environ.get("TAIL_AB_ROUNDS", "3"))
    for rnd in range(rounds):   # variants interleaved: box drift hits all of them alike
        for name, env in VARIANTS.items():
            e = dict(os.environ, GRAFT_ROOT=root, **env)
            p = subprocess.run([sys.executable, "-c", CHILD] + ks, env=e, capture_output=True, text=True,
                               timeout=300)
            line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(name, "FAILED", p.returncode, p.stderr[-2000:])
                sys.exit(1)
            res.setdefault(name, []).append(json.loads(line[0][7:]))
            print(rnd, name, {k: round(v["ms"], 4) for k, v in res[name][-1].items()}, flush=True)
    print("best of", rounds)
    for name, rs in res.items():
        print(f"  {name:20s}", {k: round(min(r[k]["ms"] for r in rs), 4) for k in rs[0]})
    roots = {json.dumps({k: v["root"] for k, v in r.items()}) for rs in res.values() for r in rs}
    print("data roots agree across variants:", len(roots) == 1)
    if len(roots) != 1:
        sys.exit(2)


if __name__ == "__main__":
    main()
