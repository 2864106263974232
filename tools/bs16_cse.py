"""Op counts of the bitsliced GF(2^16) butterfly networks (tools/bs16_netstat
output) under four signal-sharing schemes, per wave of the k = 512 encoder:

  plain  -- every row XOR-folds its input planes (3-input XORs)
  pairs  -- fixed pair sums (bitslice16.h make_sig, -DCDA_BS16_PAIR_SIGNALS): the 8 sums
            y[2i] ^ y[2i+1] formed once per butterfly, rows over 24 signals
  greedy -- Paar-style common-subexpression extraction per butterfly: the
            signal pair shared by the most rows becomes a new signal, until
            the register budget is used or no pair saves an op
  greedy3 -- the product's plan (bitslice16.h make_plan): pairs and triples
            (a triple is one 3-input XOR and drops two terms per row)

Row costs follow the kernel: base / wave rows x ^= sum of t signals ->
ceil(t / 2) ops; masked rows x ^= (sum) & m -> ceil((t - 1) / 2) + 1 ops;
wave rows run on the waves whose bit is set (weight 1/2 each).
Usage: python tools/bs16_cse.py /tmp/nets.txt [budget]"""
import collections
import math
import sys


def parse(path):
    nets = []
    for line in open(path):
        f = line.split()
        ph, layer, bf = f[0], int(f[1]), int(f[2])
        mats = []
        for tok in f[3:]:
            kind, rows = tok.split(":")
            mats.append((kind, [int(r, 16) for r in rows.split(",")]))
        nets.append((ph, layer, bf, mats))
    return nets


def row_cost(kind, t):
    if t == 0:
        return 0.0
    w = 0.5 if kind == "W" else 1.0
    return w * (math.ceil((t - 1) / 2) + 1 if kind == "L" else math.ceil(t / 2))


def cost_rows(mats, rows_terms):
    return sum(row_cost(kind, len(t)) for (kind, _), ts in zip(mats, rows_terms) for t in ts)


def plain(mats):
    rows = [[{j for j in range(16) if (r >> j) & 1} for r in m] for _, m in mats]
    return cost_rows(mats, rows), 0


def pairs(mats):
    rows = []
    for _, m in mats:
        rr = []
        for r in m:
            t = set()
            for i in range(8):
                c = (r >> (2 * i)) & 3
                if c == 1:
                    t.add(2 * i)
                elif c == 2:
                    t.add(2 * i + 1)
                elif c == 3:
                    t.add(16 + i)
            rr.append(t)
        rows.append(rr)
    return cost_rows(mats, rows) + 8, 8


def greedy(mats, budget):
    rows = [[{j for j in range(16) if (r >> j) & 1} for r in m] for _, m in mats]
    nxt, extra, made = 16, 0, 0
    while extra < budget:
        cnt = collections.Counter()
        for (kind, _), rr in zip(mats, rows):
            w = 0.5 if kind == "W" else 1.0
            for t in rr:
                s = sorted(t)
                for a in range(len(s)):
                    for b in range(a + 1, len(s)):
                        cnt[(s[a], s[b])] += w
        if not cnt:
            break
        best, base = None, cost_rows(mats, rows)
        for (a, b), _c in cnt.most_common(12):
            trial = [[(t - {a, b}) | {nxt} if a in t and b in t else t for t in rr] for rr in rows]
            gain = base - cost_rows(mats, trial) - 1
            if best is None or gain > best[0]:
                best = (gain, trial)
        if best is None or best[0] <= 0:
            break
        rows = best[1]
        nxt += 1
        extra += 1
        made += 1
    return cost_rows(mats, rows) + made, made


def greedy3(mats, budget):
    """The product's plan (bitslice16.h make_plan): pairs AND triples of
    signals, the set saving the most ops over all rows each time."""
    import itertools
    rows = [[{j for j in range(16) if (r >> j) & 1} for r in m] for _, m in mats]
    kinds = [k for k, _ in mats]
    nxt = 16
    for _ in range(budget):
        gain = collections.Counter()
        for k, rr in zip(kinds, rows):
            for t in rr:
                n = len(t)
                if n < 2:
                    continue
                d2 = row_cost(k, n) - row_cost(k, n - 1)
                d3 = row_cost(k, n) - row_cost(k, n - 2) if n >= 3 else 0
                s = sorted(t)
                if d2 > 0:
                    for c in itertools.combinations(s, 2):
                        gain[c] += d2
                if d3 > 0:
                    for c in itertools.combinations(s, 3):
                        gain[c] += d3
        if not gain:
            break
        best, g = max(gain.items(), key=lambda x: x[1])
        if g <= 1:
            break
        bs = set(best)
        rows = [[(t - bs) | {nxt} if bs <= t else t for t in rr] for rr in rows]
        nxt += 1
    return cost_rows(mats, rows) + (nxt - 16), nxt - 16


def main():
    nets = parse(sys.argv[1])
    budget = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    tot = collections.defaultdict(float)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for ph, layer, bf, mats in nets:
        for name, fn in (("plain", plain), ("pairs", pairs), ("greedy", lambda m: greedy(m, budget)),
                         ("greedy3", lambda m: greedy3(m, budget))):
            c, _ = fn(mats)
            tot[name] += c
            per[ph][name] += c
    for ph, d in per.items():
        print(f"{ph:9s} " + "  ".join(f"{k} {v:7.0f}" for k, v in d.items()))
    print("total     " + "  ".join(f"{k} {v:7.0f}" for k, v in tot.items()),
          f"  greedy vs pairs {tot['greedy'] / tot['pairs'] - 1:+.1%}, greedy3 {tot['greedy3'] / tot['pairs'] - 1:+.1%} (budget {budget} signals)")


if __name__ == "__main__":
    main()
