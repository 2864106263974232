#!/usr/bin/env python3
"""Benchmark: EDS+DAH squares/s on MI355X (BASELINE.json metric).

One step = the whole hot path (ODS -> EDS -> 4k NMT roots -> data root) over
config 4's fixed batch of 1 024 random-namespace k = 128 squares split over
the ranks (rank g: squares [g*1024/N, (g+1)*1024/N); `--batch` overrides the
per-rank count), inputs already resident in HBM, ODS in Q0 of the EDS arena
(cda_extend_dah_inplace_device).  No collective on the data path (SURVEY.md
8(e)); the total work is fixed as N grows -> "scaling": "strong".  N > 1:
under torch.distributed.run, or `--gpus N` alone (this script then starts the
N rank processes itself; launch_mode / spawn_ranks).
Timing: W untimed steps, then K steps bracketed by barrier + synchronize, max
over ranks.  Rank 0 prints one JSON line.

Extra fields: per-stage HIP-event times and rooflines, single-square latency
(k=128, config 2), k=512 single square (config 3, GF(2^16)), and the CPU
baseline (oracle/cda_oracle.c "port", same rsmt2d structure, host threads).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))

PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: 8 TB/s spec
PEAK_VALU_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T lane-slots/s
# SHA-256 compression on gfx950 as compiled: 1384 VALU
# instructions = 572 v_alignbit + 236 v_add3 (half rate, 2 issue slots each)
# + 350 v_bitop3 + 123 v_add + 93 v_lshrrev (full rate) = 2182 issue slots.
# The roofline counts issue slots (the half-rate ops are inherent to SHA-256
# on this ISA); `achieved_instr` reports the raw instruction rate.
SHA_INSTR = 1384
SHA_SLOTS = 2182
# Achievable ceilings (measured, not spec): tools/sha_probe.hip runs the same
# sha_compress stream on registers only -- 28.45 G compressions/s at 4
# waves/SIMD (profiles/r01f_sha_probe.txt), because gfx950 issues a mixed
# half-rate / full-rate stream at about the half rate (64 lane-ops/clk/CU,
# profiles/r01f_valu_probe.txt "alignbit+xor"); HBM 6.29 TB/s float4 copy
# (MI355X_MICROARCH.md).  Reported beside the spec peak as `achievable`.
ACHIEVABLE_SHA_COMP_S = 28.453e9
CONFIG5_TIMEOUT_S = float(os.environ.get("CDA_CONFIG5_TIMEOUT_S", "180"))
ACHIEVABLE_VALU_TOPS = ACHIEVABLE_SHA_COMP_S * SHA_SLOTS / 1e12
ACHIEVABLE_HBM_GBS = 6290.0
SHARE = 512
CONFIG4_SQUARES = 1024     # BASELINE.json configs[3]: 1024 independent k=128 squares over 1/2/4/8 GPUs


def compressions(k: int) -> dict:
    W = 2 * k
    return {
        "nmt_leaves": 9 * W * W,                 # 542-B leaf message = 9 blocks, one per EDS cell
        "nmt_levels": 3 * 2 * W * (W - 1),      # 181-B node message = 3 blocks
        "data_root": 2 * 2 * W + 2 * (2 * W - 1),
    }


def rs_bytes(k: int) -> int:
    return 4 * k * k * SHARE                     # ODS read + 3 parity quadrants written


# nominal 1 700 int32 VALU lane-ops per SHA-256 compression
# (48 schedule steps x 12 + 64 rounds x 17 + 8, rounded up), deduplicated
# compressions C(k) = 9*4k^2 + 3*4k(2k-1) + 2*4k + 2*(4k-1).  The peak is the
# guide's 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T (SURVEY's 39.3 T
# assumes 64 lanes per CU, half the guide's figure).
ALG_LANE_OPS_PER_COMPRESSION = 1700


def survey_compressions(k: int) -> int:
    return 9 * 4 * k * k + 3 * 4 * k * (2 * k - 1) + 2 * 4 * k + 2 * (4 * k - 1)


def combined_ceiling(k: int) -> float:
    """SURVEY 8(d) 'Combined': squares/s per GPU = 1 / (B_RS / 8 TB/s +
    C(k) * 1700 / 78.6 T), the serial sum of the RS HBM floor and the SHA-256
    VALU floor."""
    return 1.0 / (rs_bytes(k) / (PEAK_HBM_GBS * 1e9)
                  + survey_compressions(k) * ALG_LANE_OPS_PER_COMPRESSION / (PEAK_VALU_TOPS * 1e12))


def shard(rank: int, world: int, per_rank: int) -> range:
    """Config 4 (BASELINE.json configs[3]): square indexes of
    one rank.  Squares are independent, so rank g takes [g*B, (g+1)*B) with
    B = 1024 // world: the 1024 squares (seeds 0..1023) of the config split
    over the ranks, no data-path collective."""
    return range(rank * per_rank, (rank + 1) * per_rank)


def time_region(step, steps: int, sync, world: int, reduce_max=None, barrier=None) -> float:
    """The bench contract's timed region: barrier + sync, `steps` calls of
    step(), sync + barrier, then the MAX of the elapsed time over ranks
    (reduce_max(seconds) -> seconds; identity at world == 1)."""
    if world > 1 and barrier:
        barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1 and barrier:
        barrier()
    el = time.perf_counter() - t0
    if world > 1 and reduce_max:
        el = reduce_max(el)
    return el


def golden_config4():
    """tests/golden/config4_k128.json (oracle digests of squares 0..127) merged
    with config4_k128_rest.json (data roots of squares 128..1023; both by
    oracle/gen_config4.py), so every rank's shard is checked; or None."""
    p = os.path.join(ROOT, "tests", "golden", "config4_k128.json")
    try:
        with open(p) as f:
            g = json.load(f)
        rest = os.path.join(ROOT, "tests", "golden", "config4_k128_rest.json")
        if os.path.exists(rest):
            with open(rest) as f:
                g["squares"].update(json.load(f)["squares"])
        return g
    except OSError:
        return None


def golden_k512():
    p = os.path.join(ROOT, "tests", "golden", "k512.json")
    try:
        with open(p) as f:
            return json.load(f)["squares"]
    except (OSError, KeyError):
        return None


def host_buffer_rates(ctx, k: int, n: int = 16, reps: int = 5) -> dict:
    """The drop-in boundary with host buffers: squares/s of
    cda_extend_dah_batch when the ODS comes from and the EDS, roots and data
    roots go back to host memory (PCIe inside, never the headline), and the
    ProcessProposal latency from the block's host txs
    (cda_construct_extend_dah: square construction + extension + DAH).
    Host buffers are allocated once and reused, as a node reuses them (fresh
    pages would add the kernel's first-touch faults to every call)."""
    import ctypes as C

    import numpy as np

    from celestia_da import blobfactory, square as gsq, testfactory
    from celestia_da._lib import ptr
    W = 2 * k
    ods = np.ascontiguousarray(np.stack([testfactory.random_square(k, 5000 + i) for i in range(n)]))
    eds = np.ones((n, W * W * SHARE), dtype=np.uint8)
    rows = np.ones((n, W * 90), dtype=np.uint8)
    cols = np.ones((n, W * 90), dtype=np.uint8)
    roots = np.ones((n, 32), dtype=np.uint8)
    status = np.zeros(n, dtype=np.int32)
    st = status.ctypes.data_as(C.POINTER(C.c_int32))

    def run(with_eds, m=n):
        ctx.check(ctx.lib.cda_extend_dah_batch(ctx.h, ptr(ods[:m]), k, m, ptr(eds[:m]) if with_eds else None,
                                               ptr(rows[:m]), ptr(cols[:m]), ptr(roots[:m]), st))

    def med(f):
        f()
        t = []
        for _ in range(reps):
            a = time.perf_counter()
            f()
            t.append(time.perf_counter() - a)
        return sorted(t)[reps // 2]

    full = med(lambda: run(True))
    only_roots = med(lambda: run(False))
    one = med(lambda: run(True, 1))
    one_roots = med(lambda: run(False, 1))
    txs = blobfactory.full_block(1, 128)
    pp = med(lambda: gsq.construct_extend_dah(txs, 128, ctx=ctx))
    # the C-ABI call alone, with the txs already in one flat buffer (what a cgo
    # caller passes) and output buffers reused
    buf, off = gsq._flatten(txs)
    wm = 2 * 128
    prow = np.empty(wm * 90, dtype=np.uint8)
    pcol = np.empty(wm * 90, dtype=np.uint8)
    proot = np.empty(32, dtype=np.uint8)
    kk, nk = C.c_uint32(), C.c_uint32()
    kept = (C.c_uint32 * len(txs))()

    def pp_call():
        ctx.check(ctx.lib.cda_construct_extend_dah(ctx.h, ptr(buf), gsq._u64p(off), len(txs), 128, 64,
                                                   gsq._lib.CDA_SQUARE_CONSTRUCT, None, 0, ptr(prow), ptr(pcol),
                                                   prow.size, ptr(proot), C.byref(kk), kept, C.byref(nk)))

    pp_c = med(pp_call)
    return {"k": k, "squares": n,
            "eds_to_host_squares_per_s": n / full,
            "pcie_gb_per_s": n * (k * k + 3 * k * k) * SHARE / full / 1e9,
            "roots_only_squares_per_s": n / only_roots,
            "one_square_eds_to_host_ms": 1e3 * one, "one_square_roots_only_ms": 1e3 * one_roots,
            "process_proposal_ms": 1e3 * pp, "process_proposal_c_abi_ms": 1e3 * pp_c,
            "note": "cda_extend_dah_batch with reused host buffers: H2D ODS, D2H of the three parity quadrants "
                    "(the host copies Q0 from the ODS) overlapping the hashing, D2H roots; pcie_gb_per_s counts "
                    "ODS in + parity out; process_proposal_ms = cda_construct_extend_dah on a full k=128 block of "
                    "blob txs (host txs -> data root, roots back to the host) through the Python wrapper (which "
                    "also flattens the txs and builds the root lists); process_proposal_c_abi_ms = the C call alone "
                    "on an already flat tx buffer"}


def host_pipeline_rates(ctx, k: int, d_ods, d_eds, idx, reps: int = 3) -> dict:
    """Config 4 through the drop-in boundary with host buffers (VERDICT r3
    item 3; pkg/da/data_availability_header.go:65-75 takes host shares and
    returns a host EDS): all of this rank's squares through ONE
    cda_extend_dah_batch call from page-locked host buffers, which the library
    runs as a chunk pipeline (H2D of chunk i+1, compute of chunk i and D2H of
    chunk i-1 on three streams; engine.hip host_pipeline).  Reports roots-only
    and EDS-returned rates and the PCIe GB/s each moves, beside the line rates
    of plain pinned copies of the same bytes measured in the same run; every
    data root (and the EDS digests the fixture holds) is checked against the
    oracle fixtures.  PCIe inside: never the headline."""
    import ctypes as C
    import hashlib

    import numpy as np
    import torch

    from celestia_da._lib import ptr
    n = d_ods.shape[0]
    W = 2 * k
    ods_b, eds_b = k * k * SHARE, W * W * SHARE
    h_ods = torch.empty((n, ods_b), dtype=torch.uint8, pin_memory=True)
    h_ods.copy_(d_ods.view(n, -1))
    h_eds = torch.empty((n, eds_b), dtype=torch.uint8, pin_memory=True)
    rows = np.empty((n, W * 90), dtype=np.uint8)
    cols = np.empty((n, W * 90), dtype=np.uint8)
    roots = np.empty((n, 32), dtype=np.uint8)
    status = np.zeros(n, dtype=np.int32)
    st = status.ctypes.data_as(C.POINTER(C.c_int32))

    def tptr(t):   # a pinned tensor as the uint8_t* the C ABI takes
        return C.cast(C.c_void_p(t.data_ptr()), C.POINTER(C.c_ubyte))

    def run(with_eds):
        ctx.check(ctx.lib.cda_extend_dah_batch(ctx.h, tptr(h_ods), k, n, tptr(h_eds) if with_eds else None,
                                               ptr(rows), ptr(cols), ptr(roots), st))

    def med(f):
        f()
        t = []
        for _ in range(reps):
            a = time.perf_counter()
            f()
            t.append(time.perf_counter() - a)
        return sorted(t)[len(t) // 2]

    # line rates: plain pinned copies of the same bytes (one direction at a time)
    dev = d_ods.device

    def h2d():
        d_ods.view(n, -1).copy_(h_ods, non_blocking=True)
        torch.cuda.synchronize(dev)

    par = n * 3 * ods_b   # the three parity quadrants (the host copies Q0 itself)

    def d2h():
        h_eds.view(-1)[:par].copy_(d_eds.view(-1)[:par], non_blocking=True)
        torch.cuda.synchronize(dev)

    s_up, s_down = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def both():   # the pipeline's mix: ODS up and parity down at once, on two streams
        with torch.cuda.stream(s_up):
            d_ods.view(n, -1).copy_(h_ods, non_blocking=True)
        with torch.cuda.stream(s_down):
            h_eds.view(-1)[:par].copy_(d_eds.view(-1)[:par], non_blocking=True)
        torch.cuda.synchronize(dev)

    t_h2d, t_d2h, t_both = med(h2d), med(d2h), med(both)
    t_roots = med(lambda: run(False))
    t_eds = med(lambda: run(True))
    g = golden_config4()

    def check_roots_and_eds(eds_of):
        checked = matched = eds_checked = eds_matched = 0
        if g and g.get("k") == k:
            for j, i in enumerate(idx[:n]):
                want = g["squares"].get(str(i))
                if want is None:
                    continue
                checked += 1
                matched += int(roots[j].tobytes().hex() == want["data_root"])
                if "eds_sha256" in want and eds_checked < 8:
                    eds_checked += 1
                    eds_matched += int(hashlib.sha256(eds_of(j)).hexdigest() == want["eds_sha256"])
        assert int(np.abs(status).sum()) == 0, "push-order status set on ordered input"
        assert matched == checked and eds_matched == eds_checked, (matched, checked, eds_matched, eds_checked)
        return {"data_roots_checked": checked, "data_roots_matched": matched,
                "eds_digests_checked": eds_checked, "eds_digests_matched": eds_matched}

    par_check = check_roots_and_eds(lambda j: h_eds[j].numpy().tobytes())
    # packed parity (CDA_EDS_PARITY): the caller keeps Q0 (its own shares), the
    # device packs each chunk's parity and returns it in one linear copy; the
    # buffer reuses h_eds's pinned storage
    from celestia_da import _lib as _L
    from celestia_da.da import unpack_parity
    h_par = h_eds.view(-1)[:n * 3 * ods_b].view(n, 3 * ods_b)

    def run_packed():
        ctx.check(ctx.lib.cda_extend_dah_batch_ex(ctx.h, tptr(h_ods), k, n, tptr(h_par), _L.CDA_EDS_PARITY,
                                                  ptr(rows), ptr(cols), ptr(roots), st))

    t_par = med(run_packed)
    packed_check = check_roots_and_eds(lambda j: unpack_parity(h_ods[j].numpy(), h_par[j].numpy().reshape(-1, SHARE))
                                       .tobytes())
    h2d_line, d2h_line = n * ods_b / t_h2d / 1e9, par / t_d2h / 1e9
    roots_gbs, eds_gbs = n * ods_b / t_roots / 1e9, par / t_eds / 1e9
    return {"k": k, "squares": n,
            "roots_only_squares_per_s": n / t_roots, "roots_only_h2d_gb_per_s": roots_gbs,
            "h2d_line_gb_per_s": h2d_line, "roots_only_frac_of_h2d_line": roots_gbs / h2d_line,
            "eds_to_host_squares_per_s": n / t_eds, "eds_d2h_gb_per_s": eds_gbs,
            "d2h_line_gb_per_s": d2h_line, "eds_frac_of_d2h_line": eds_gbs / d2h_line,
            "bidir_line_squares_per_s": n / t_both, "eds_frac_of_bidir_line": t_both / t_eds,
            "packed_parity_squares_per_s": n / t_par, "packed_parity_d2h_gb_per_s": par / t_par / 1e9,
            "packed_frac_of_bidir_line": t_both / t_par, "packed_frac_of_d2h_line": t_d2h / t_par,
            "parity": par_check, "parity_packed": packed_check,
            "note": "one cda_extend_dah_batch call over the rank's squares from page-locked host buffers "
                    "(torch pin_memory): ODS up, roots (and with the EDS: the three parity quadrants) down; "
                    "the library pipelines 32-square chunks over three streams; line rates = plain pinned "
                    "copies of the same bytes in the same run, one direction at a time; bidir line = both copies at once "
                    "on two streams (the pipeline's own mix of ODS up and parity down); packed_parity = "
                    "cda_extend_dah_batch_ex(CDA_EDS_PARITY): the caller keeps Q0 (its shares), parity packed on the "
                    "device and returned in one linear copy per chunk, EDS digests checked on the reassembled square"}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def stage_report(st: dict, k: int, batch: int, inplace: bool = False, steps: int = 0) -> dict:
    """Per-stage roofline records.  With `steps` (> 0) the stage may run as
    several launches per step (the chunked batch pipeline): `avg_ms` is then
    the stage's time per step and the work is the whole batch's; otherwise one
    launch covers `batch` squares."""
    out = {}
    comp = compressions(k)
    for name, (ms, n) in st.items():
        if n == 0:
            continue
        avg = ms / (steps if steps > 0 else n)
        rec = {"avg_ms": avg, "launches": n}
        if steps > 0:
            rec["launches_per_step"] = n / steps
        if name in comp:
            # compressions x 1 700 nominal int32 lane-ops against
            # the 78.6 T VALU peak; the compiled-issue-slot view beside it
            c = comp[name] * batch
            rec.update(bound="valu", achieved=c * ALG_LANE_OPS_PER_COMPRESSION / (avg * 1e-3) / 1e12,
                       peak=PEAK_VALU_TOPS, unit="T int32 lane-ops/s (8(d): 1700 per SHA-256 compression)",
                       compressions=c, compressions_per_s=c / (avg * 1e-3),
                       frac_issue_slots=c * SHA_SLOTS / (avg * 1e-3) / 1e12 / PEAK_VALU_TOPS)
        elif name in ("rs_q0", "rs_q3"):
            # rs_q0: read ODS, write Q0|Q1|Q2 (4 k^2 shares); rs_q3: read Q2, write Q3 (2 k^2 shares)
            # (in place there is no Q0 copy: read Q0, write Q1|Q2 = 3 k^2 shares)
            # (no separate Q3 stage recorded: rs_q0 is the whole RS)
            whole = name == "rs_q0" and st.get("rs_q3", (0.0, 0))[1] == 0
            byt = ((3 if inplace else 4) + (2 if whole else 0) if name == "rs_q0" else 2) * k * k * SHARE * batch
            rec.update(bound="hbm", achieved=byt / (avg * 1e-3) / 1e9, peak=PEAK_HBM_GBS, unit="GB/s")
        if "achieved" in rec:
            rec["frac"] = rec["achieved"] / rec["peak"]
            if rec["bound"] == "valu":   # against the measured SHA-256 issue ceiling (tools/sha_probe.hip)
                rec["frac_of_achievable"] = rec["compressions_per_s"] / ACHIEVABLE_SHA_COMP_S
            else:
                rec["frac_of_achievable"] = rec["achieved"] / ACHIEVABLE_HBM_GBS
        out[name] = rec
    return out


PMC_SUMMARY = os.environ.get("CDA_PMC_SUMMARY", "")


def load_pmc(stage: str, field: str = "hbm_bytes_per_launch"):
    """A per-launch figure of `stage` from the committed rocprofv3 PMC summary
    (profiles/*_pmc.json, written by tools/pmc_summary.py from separate --pmc
    passes of this bench: FETCH_SIZE / WRITE_SIZE -> HBM bytes, SQ_INSTS_VALU
    ...), else None.  The newest summary (by round tag) is used unless
    CDA_PMC_SUMMARY names one."""
    import glob
    # newest by round tag (r01_ < r01b_ < ... < r02_ < r02b_ < r02c_ sort by
    # name; file times depend on how the tree was copied)
    files = [PMC_SUMMARY] if PMC_SUMMARY else sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            d = json.load(f)
        return d.get(stage, {}).get(field)
    except Exception:
        return None


def load_traffic(stage: str):
    return load_pmc(stage, "hbm_bytes_per_launch")


def alg_bytes_per_square(kernel: str, k: int) -> int:
    """Algorithmic HBM bytes per square of each hot kernel:
    every input byte read once and every output byte written once.
      rs_gf8_bs / rs_gf16: 8(d)'s B_RS = 4 k^2 512 (Q0 read, Q1|Q2|Q3 written)
      nmt_leaves: the EDS read once (W^2 512) + one 96-B leaf slot per cell
      nmt_levels: every level reads its children and writes its parents,
                  2W trees x (2W - 2) child slots read + (W - 1) parents, 96 B"""
    W = 2 * k
    if kernel in ("rs_gf8_bs", "rs_gf16"):
        return rs_bytes(k)
    if kernel == "nmt_leaves":
        return W * W * (SHARE + 96)
    if kernel == "nmt_levels":
        return 2 * W * ((2 * W - 2) + (W - 1)) * 96
    raise KeyError(kernel)


def traffic_report(k: int, squares_per_step: int) -> dict:
    """Measured HBM bytes (PMC summary, FETCH_SIZE x 2 + WRITE_SIZE, separate
    rocprofv3 passes of a fixed-shape run: tools/profile_round3.sh) per
    square and per step of each hot kernel, and their ratio to the
    algorithmic bytes.  Reproducible from the summary alone:
    hbm_bytes_per_square = hbm_bytes_per_launch x launches_per_step /
    squares_per_step of the profiled run (its _config)."""
    out = {}
    cfg = load_pmc("_config", "k128" if k == 128 else f"k{k}") or {}
    for kern in ("rs_gf8_bs" if k <= 128 else "rs_gf16", "nmt_leaves", "nmt_levels"):
        per_sq = load_pmc(kern, f"hbm_bytes_per_square_k{k}")
        if per_sq is None:
            continue
        alg = alg_bytes_per_square(kern, k)
        out[kern] = {"hbm_bytes_per_square": per_sq, "traffic_per_step": per_sq * squares_per_step,
                     "algorithmic_bytes_per_square": alg, "traffic_ratio": per_sq / alg,
                     "profiled_shape": cfg}
    return out


def cpu_threads(requested: int = 0) -> tuple:
    """(threads used, host CPUs visible).  SURVEY 8(d) asks for all host
    cores: every CPU in this process's affinity mask, capped by
    OMP_NUM_THREADS when the environment sets it (the GPU box grants one
    GPU's job 16 CPUs and sets OMP_NUM_THREADS=16; nproc there shows the
    whole machine)."""
    host = len(os.sched_getaffinity(0))
    if requested:
        return requested, host
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(host, cap) if cap > 0 else host), host


def cpu_baseline(k: int, seconds: float, threads: int, runs: int = 5):
    """CPU restatement (NOT the reference: Go is absent on both machines), timed
    as SURVEY 8(d) asks: 1 warm-up, then `runs` samples of ~seconds/runs each,
    the median squares/s reported."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle
    threads, host = cpu_threads(threads)
    ods = coracle.random_square(k, 0)
    coracle.cpu_baseline(ods, threads)          # warm-up
    rates, total_n, total_t = [], 0, 0.0
    for _ in range(runs):
        n, t0 = 0, time.perf_counter()
        while True:
            coracle.cpu_baseline(ods, threads)
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds / runs or n >= 1000:
                break
        rates.append(n / el)
        total_n += n
        total_t += el
    rates.sort()
    return {"value": rates[len(rates) // 2], "unit": "squares/s", "cores": threads, "kind": "port",
            "label": "CPU restatement, not reference", "host_cpus": host, "cpu_model": cpu_model(),
            "runs": rates,
            "sample": f"median of {runs} runs, {total_n} squares k={k} in {total_t:.1f}s (oracle/cda_oracle.c "
                      f"oracle_cpu_baseline: rsmt2d structure, every cell hashed in its row and its column tree, "
                      f"SHA-NI + AVX2 PSHUFB Leopard as in Go's amd64 assembly; {threads} threads of {host} "
                      f"visible CPUs, {cpu_model()})"}


def config5(ctx, dev, rank: int, world: int, k: int, iters: int = 5, emit=None) -> dict:
    """Config 5 timing: one k x k square split over `world`
    GPUs, by both drivers of the same kernels: the library's own RCCL
    communicator (cda_comm_init + cda_extend_dah_split, what a cgo host uses)
    and torch.distributed (celestia_da.dist.extend_dah_split).  Reports ms per
    square (max over ranks); rank 0 checks both results against its
    single-GPU extend_dah of the same square."""
    import torch
    import torch.distributed as dist

    from celestia_da import _lib
    from celestia_da import dist as cdist
    from celestia_da import testfactory

    ods = testfactory.random_square(k, 0).reshape(k, k, SHARE)
    R = k // world
    mine = torch.from_numpy(ods[rank * R:(rank + 1) * R].copy()).to(dev)
    on = dev if dist.get_backend() == "nccl" else "cpu"

    def max_over_ranks(x: float, bad: int):
        el = torch.tensor([x, float(bad)], dtype=torch.float64, device=on)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el[0].item()), el[1].item() > 0

    def timed(run):
        run()                                   # warm-up
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            res = run()
        torch.cuda.synchronize(dev)
        dist.barrier()
        return time.perf_counter() - t0, res

    out = {"k": k, "gpus": world, "all_to_all_bytes_per_rank": R * (2 * k) * SHARE * (world - 1) // world}
    W = 2 * k
    ref = None
    if rank == 0:
        e = torch.empty(W * W * SHARE, dtype=torch.uint8, device=dev)
        r1 = torch.empty(W * 90, dtype=torch.uint8, device=dev)
        c1 = torch.empty(W * 90, dtype=torch.uint8, device=dev)
        g1 = torch.empty(32, dtype=torch.uint8, device=dev)
        o = torch.from_numpy(ods.reshape(-1, SHARE).copy()).to(dev)
        ctx.extend_dah_device(o.data_ptr(), k, 1, e.data_ptr(), r1.data_ptr(), c1.data_ptr(), g1.data_ptr(),
                              None, torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        ref = (r1.view(W, 90), c1.view(W, 90), g1)
        out["data_root"] = g1.cpu().numpy().tobytes().hex()
        del e, o

    def matches(res) -> bool:
        rows, cols, root, err = res
        return bool(torch.equal(ref[2], root) and torch.equal(ref[0], rows) and torch.equal(ref[1], cols)
                    and int(err.item()) == 0xFFFFFFFF)

    # (1) torch.distributed collectives (every rank enters every collective even
    # if a local step fails)
    ops = cdist.GpuSplitOps(ctx, dev)
    errors = []
    el, res = timed(lambda: cdist.extend_dah_split(mine, k, ops, rank, world, on_error=errors.append))
    el, bad = max_over_ranks(el, len(errors))
    if bad:
        out["torch_distributed"] = {"error": repr(errors[0]) if errors else "failed on another rank"}
    else:
        out["torch_distributed"] = {"ms_per_square": 1e3 * el / iters, "squares_per_s": iters / el}
        if rank == 0:
            out["torch_distributed"]["matches_single_gpu"] = matches(res[2])
    if emit:
        emit(out)   # a hang in the next leg keeps this one's result
    # (2) library RCCL communicator
    try:
        uid = torch.zeros(128, dtype=torch.uint8, device=on)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(_lib.comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, src=0)
        c = _lib.Context(dev.index)
        c.comm_init(rank, world, bytes(uid.cpu().numpy()))
        comm_rank, comm_world = c.comm_size()
        el, res = timed(lambda: cdist.extend_dah_split_rccl(c, mine, k, rank, world))
        el, bad = max_over_ranks(el, 0)
        out["library_rccl"] = {"ms_per_square": 1e3 * el / iters, "squares_per_s": iters / el,
                               "communicator_ranks": comm_world}
        if rank == 0:
            out["library_rccl"]["matches_single_gpu"] = matches(res[1])
        c.comm_destroy()
        c.close()
    except Exception as ex:  # report, keep the torch.distributed leg
        out["library_rccl"] = {"error": f"{type(ex).__name__}: {ex}"}
    return out


def config5_isolated(world: int, timeout_s: float) -> dict:
    """Run config5() in a child of this rank (same RANK / WORLD_SIZE /
    LOCAL_RANK, MASTER_PORT + 7 for the children's own process group) and
    return rank 0's result; a hang is killed at timeout_s, a crash is reported.
    Every rank waits for its own child only, so no collective of the parent
    group depends on the children."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env["MASTER_PORT"] = str(int(os.environ.get("MASTER_PORT", "29517")) + 7)
    # under torch.distributed.run the env:// rendezvous would join the launch
    # agent's store (on the parent's port); the children's rank 0 hosts its own
    env["TORCHELASTIC_USE_AGENT_STORE"] = "False"
    env.setdefault("RANK", "0")
    env.setdefault("WORLD_SIZE", str(world))
    env.setdefault("LOCAL_RANK", "0")
    cmd = [sys.executable, os.path.abspath(__file__), "--config5-child", "--no-cpu"]
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    res = {}
    try:
        out, err = p.communicate(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        p.kill()
        out, err = p.communicate()
        res["error"] = f"no result after {timeout_s} s (collective hang?)"
    for ln in out.splitlines():   # the legs reported so far (rank 0's child)
        if ln.startswith("CONFIG5 "):
            res.update(json.loads(ln[8:]))
    if p.returncode not in (0, None) and "error" not in res and p.returncode != -9:
        res["error"] = f"config-5 child exited with {p.returncode}"
    if "error" in res:   # the child's last words, minus the runtime's noise
        tail = [ln for ln in err.splitlines() if "amdgpu.ids" not in ln and "hostname of the client" not in ln]
        res["child_stderr_tail"] = "\n".join(tail)[-600:]
    return res or {"rank_result": "only rank 0 reports"}


def square_construction(ctx, dev, stream, max_ss: int = 128, reps: int = 20) -> dict:
    """go-square square.Construct on a full k=128 block of
    blob txs (celestia_da.blobfactory.full_block), then the fused path txs ->
    data root.  Host layout planning and the device share writer are timed
    separately; the writer's bytes are payload read + k*k*512 written."""
    import ctypes as C

    import torch

    from celestia_da import blobfactory
    from celestia_da import square as gsq

    txs = blobfactory.full_block(1, max_ss)
    buf, off = gsq._flatten(txs)
    L = ctx.lib
    k = C.c_uint32()
    plan_t = []
    for _ in range(reps):
        a = time.perf_counter()
        ctx.check(L.cda_square_layout(ctx.h, gsq.ptr(buf), gsq._u64p(off), len(txs), max_ss, 64, 0, C.byref(k),
                                      None, None, None, 0, None))
        plan_t.append(time.perf_counter() - a)
    k = k.value
    d_txs = torch.zeros(buf.size + 16, dtype=torch.uint8, device=dev)
    d_txs[:buf.size] = torch.from_numpy(buf).to(dev)
    d_ods = torch.empty(max_ss * max_ss * SHARE, dtype=torch.uint8, device=dev)
    W = 2 * k
    d_eds = torch.empty(W * W * SHARE, dtype=torch.uint8, device=dev)
    d_rows = torch.empty(W * 90, dtype=torch.uint8, device=dev)
    d_cols = torch.empty(W * 90, dtype=torch.uint8, device=dev)
    d_root = torch.empty(32, dtype=torch.uint8, device=dev)
    kk = C.c_uint32()

    def construct():
        ctx.check(L.cda_square_construct_device(ctx.h, gsq.ptr(buf), gsq._u64p(off), len(txs), d_txs.data_ptr(),
                                                max_ss, 64, 0, d_ods.data_ptr(), d_ods.numel(), C.byref(kk), None,
                                                None, stream))

    construct()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    wall, full = [], []
    for e0, e1 in ev:
        a = time.perf_counter()
        e0.record()
        construct()
        e1.record()
        torch.cuda.synchronize(dev)
        wall.append(time.perf_counter() - a)
    dev_ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)[reps // 2]
    for _ in range(reps):
        a = time.perf_counter()
        construct()
        ctx.extend_dah_device(d_ods.data_ptr(), k, 1, d_eds.data_ptr(), d_rows.data_ptr(), d_cols.data_ptr(),
                              d_root.data_ptr(), None, stream)
        torch.cuda.synchronize(dev)
        full.append(time.perf_counter() - a)
    payload = int(off[-1])
    moved = payload + k * k * SHARE
    return {"k": k, "n_txs": len(txs), "tx_bytes": payload,
            "plan_ms_host": 1e3 * sorted(plan_t)[reps // 2],
            "writer_ms_device": dev_ms, "writer_gb_per_s": moved / (dev_ms * 1e-3) / 1e9,
            "construct_ms_wall": 1e3 * sorted(wall)[reps // 2],
            "txs_to_data_root_ms_wall": 1e3 * sorted(full)[reps // 2],
            "data_root": d_root.cpu().numpy().tobytes().hex()}


def eds_repair(ctx, k: int = 128, reps: int = 5) -> dict:
    """rsmt2d ExtendedDataSquare.Repair on the GPU
    (cda_repair_device on an HBM-resident square, and cda_repair with host
    buffers, PCIe inside) for two
    erasure patterns of one random k=128 square: the whole original quadrant
    lost (one sweep: every row decodes from its parity half), and a random
    half of every row lost (rows alone cannot all finish; columns complete
    them).  Each repaired square is checked against the extension."""
    import ctypes as C

    import numpy as np

    from celestia_da import da, testfactory
    from celestia_da._lib import ptr

    W = 2 * k
    ods = testfactory.random_square(k, 7)
    sq = da.extend_shares(ods)
    dah = da.new_data_availability_header(sq)
    full = np.ascontiguousarray(sq.array())
    rows = np.frombuffer(b"".join(dah.row_roots), dtype=np.uint8)
    cols = np.frombuffer(b"".join(dah.column_roots), dtype=np.uint8)
    rng = np.random.default_rng(5)
    pats = {"q0_lost": np.ones((W, W), np.uint8), "half_of_every_row_lost": np.ones((W, W), np.uint8)}
    pats["q0_lost"][:k, :k] = 0
    for r in range(W):
        pats["half_of_every_row_lost"][r, rng.choice(W, k, replace=False)] = 0
    import torch

    out = {"k": k}
    for name, p in pats.items():
        er = np.where(p[..., None].astype(bool), full, 0).astype(np.uint8)
        host_t, dev_t = [], []
        d = torch.empty(er.size, dtype=torch.uint8, device="cuda")
        src = torch.from_numpy(er.reshape(-1)).to("cuda")
        for _ in range(reps + 1):
            e = er.copy()
            ax, ix = C.c_int32(-1), C.c_uint32(0)
            a = time.perf_counter()
            rc = ctx.lib.cda_repair(ctx.h, ptr(e), ptr(p), W, ptr(rows), ptr(cols), C.byref(ax), C.byref(ix))
            host_t.append(time.perf_counter() - a)
            ctx.check(rc)
            assert np.array_equal(e, full), "repaired square differs"
            d.copy_(src)
            torch.cuda.synchronize()
            a = time.perf_counter()
            rc = ctx.lib.cda_repair_device(ctx.h, d.data_ptr(), ptr(p), W, ptr(rows), ptr(cols), C.byref(ax),
                                           C.byref(ix))
            dev_t.append(time.perf_counter() - a)
            ctx.check(rc)
        assert np.array_equal(d.cpu().numpy().reshape(W, W, 512), full), "device-repaired square differs"
        med = lambda t: 1e3 * sorted(t[1:])[len(t[1:]) // 2]  # noqa: E731
        out[name] = {"erased_cells": int((p == 0).sum()), "ms_device": med(dev_t), "ms_host_buffers": med(host_t)}
    out["note"] = ("ms_device: cda_repair_device on an HBM-resident square (wall: pristine copy, decode sweeps, "
                   "and the final verification of every row and column -- a full NMT + re-encode pass, which also "
                   "covers rsmt2d's pre-repair sanity check; that check runs separately only on the error path); "
                   "ms_host_buffers adds the 32 MiB copies each way")
    return out


def share_proofs(ctx, k: int = 128, reps: int = 200) -> dict:
    """proof.NewShareInclusionProofFromEDS served from a
    resident square (cda_square_create keeps the EDS, every row-tree level and
    the data-root tree in HBM; each proof is index arithmetic + one gather).
    Reports the create time and the median wall time of one proof for a
    one-share range and a 2-row range (host output buffers)."""
    import numpy as np

    from celestia_da import proof as gpr
    from celestia_da import testfactory

    ods = testfactory.random_square(k, 11)
    warm = []
    for i in range(4):   # the first create also allocates the context's scratch
        a = time.perf_counter()
        sq = gpr.ResidentSquare(ods)
        warm.append(1e3 * (time.perf_counter() - a))
        if i < 3:
            sq.close()
    out = {"k": k, "create_ms_wall_first": warm[0], "create_ms_wall": sorted(warm[1:])[1],
           "create_note": "host ODS -> resident EDS + every row-tree level + data-root tree (PCIe copy included)"}
    try:
        for name, (s, e) in {"one_share": (5 * k + 3, 5 * k + 4), "two_rows": (7 * k + 10, 9 * k - 10)}.items():
            ns = bytes(np.asarray(ods[s])[:29])
            sq.share_proof(ns, s, e)
            t = []
            for _ in range(reps):
                b = time.perf_counter()
                sq.share_proof(ns, s, e)
                t.append(time.perf_counter() - b)
            out[name] = {"shares": e - s, "us_wall": 1e6 * sorted(t)[len(t) // 2]}
    finally:
        sq.close()
    return out


def blob_commitments(ctx, dev, stream, n_blocks: int = 64, reps: int = 10) -> dict:
    """inclusion.CreateCommitment for every blob of
    n_blocks full k=128 blocks (blobfactory.full_block_blobs), blob bytes
    resident in HBM (cda_blob_commitments_device); plus one block's blobs
    (ProcessProposal's ValidateBlobTx sweep) as a latency figure.  Roofline:
    SHA-256 issue slots (9 compressions per share, 3 per NMT inner node, 2 per
    RFC-6962 node)."""
    import ctypes as C

    import numpy as np
    import torch

    from celestia_da import blobfactory
    from celestia_da import inclusion as ginc

    def setup(blocks):
        ns, datas = [], []
        for b in blocks:
            for ns_id, data in blobfactory.full_block_blobs(100 + b, 128):
                ns.append(b"\x00" + ns_id)
                datas.append(data)
        n = len(datas)
        nsb = np.frombuffer(b"".join(ns), dtype=np.uint8).copy()
        off = np.zeros(n + 1, dtype=np.uint64)
        for i, d in enumerate(datas):
            off[i + 1] = off[i] + len(d)
        flat = np.frombuffer(b"".join(datas), dtype=np.uint8)
        d_data = torch.zeros(flat.size + 16, dtype=torch.uint8, device=dev)
        d_data[:flat.size] = torch.from_numpy(flat.copy()).to(dev)
        d_out = torch.empty(32 * n, dtype=torch.uint8, device=dev)
        comp = sum(ginc.sha256_compressions(len(d)) for d in datas)
        return n, nsb, off, d_data, d_out, comp

    def measure(n, nsb, off, d_data, d_out):
        offp = off.ctypes.data_as(C.POINTER(C.c_uint64))
        nsp = nsb.ctypes.data_as(C.POINTER(C.c_uint8))

        def run():
            ctx.check(ctx.lib.cda_blob_commitments_device(ctx.h, nsp, offp, None, n, 64, d_data.data_ptr(),
                                                          d_out.data_ptr(), stream))
        run()
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        wall = []
        for e0, e1 in ev:
            a = time.perf_counter()
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize(dev)
            wall.append(time.perf_counter() - a)
        return sorted(e0.elapsed_time(e1) for e0, e1 in ev)[reps // 2], 1e3 * sorted(wall)[reps // 2]

    n, nsb, off, d_data, d_out, comp = setup(range(n_blocks))
    ms, _ = measure(n, nsb, off, d_data, d_out)
    slots = comp * SHA_SLOTS / (ms * 1e-3) / 1e12
    n1, nsb1, off1, d1, o1, _ = setup([0])
    ms1, wall1 = measure(n1, nsb1, off1, d1, o1)
    return {"blobs": n, "blob_bytes": int(off[-1]), "ms": ms, "commitments_per_s": n / (ms * 1e-3),
            "blob_gb_per_s": int(off[-1]) / (ms * 1e-3) / 1e9,
            "roofline": {"bound": "valu", "achieved": slots, "peak": PEAK_VALU_TOPS, "unit": "T issue-slots/s",
                         "frac": slots / PEAK_VALU_TOPS, "compressions": comp},
            "one_block": {"blobs": n1, "blob_bytes": int(off1[-1]), "ms_device": ms1, "ms_wall": wall1},
            "workload": f"all blobs of {n_blocks} full k=128 blocks (CheckTx/ProcessProposal ValidateBlobTx)"}


def gather_parity(parity: dict, world: int, device) -> dict:
    """Every rank's {checked, matched} fixture counts, summed, with the
    per-rank list (rank order) -- what rank 0's line reports at N > 1."""
    import torch
    import torch.distributed as dist
    pt = torch.tensor([parity["checked"], parity["matched"]], dtype=torch.int64, device=device)
    allp = [torch.zeros_like(pt) for _ in range(world)]
    dist.all_gather(allp, pt)
    per = [[int(x[0]), int(x[1])] for x in allp]
    return {"checked": sum(c for c, _ in per), "matched": sum(m for _, m in per), "per_rank": per}


def launch_mode(gpus: int, env) -> str:
    """How `bench.py --gpus N` runs:
    - WORLD_SIZE set (torch.distributed.run or our own spawn): this process is
      one rank; WORLD_SIZE must equal --gpus, else the run is refused
      ("mismatch") instead of silently measuring another world size;
    - WORLD_SIZE unset and N == 1: one rank in this process ("inprocess");
    - WORLD_SIZE unset and N > 1: this process stays GPU-free and starts N
      rank processes itself ("spawn")."""
    if gpus < 1:
        return "mismatch"
    ws = env.get("WORLD_SIZE")
    if ws is not None and ws != "":
        return "rank" if int(ws) == gpus else "mismatch"
    return "inprocess" if gpus == 1 else "spawn"


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_commands(argv: list, gpus: int, port: int, env) -> list:
    """(argv, env) of each rank process of a self-spawned N-rank run: the same
    script and arguments, with the env:// rendezvous variables
    torch.distributed.run would set (RANK = LOCAL_RANK = g, WORLD_SIZE = N,
    MASTER_ADDR 127.0.0.1, a free MASTER_PORT)."""
    out = []
    for g in range(gpus):
        e = dict(env)
        e.update({"RANK": str(g), "LOCAL_RANK": str(g), "WORLD_SIZE": str(gpus), "LOCAL_WORLD_SIZE": str(gpus),
                  "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                  "CDA_BENCH_LAUNCHER": "bench.py"})
        out.append(([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), e))
    return out


def _exit_status(rc: int) -> int:
    return rc if rc > 0 else 128 - rc    # -N (killed by signal N) -> 128 + N, as a shell reports it


def spawn_ranks(argv: list, gpus: int, grace_s: float = 60.0) -> int:
    """Run N rank processes (children, never an exec: this parent has not
    touched the GPU and does not import torch).  Rank 0 prints the JSON line
    on the inherited stdout.  When a rank fails, the others get `grace_s` to
    finish (they may be blocked in a collective with it), then their process
    groups are killed.  Returns the first non-zero exit status, else 0."""
    import signal
    import subprocess

    def die_with_parent():   # in the child, before exec: SIGKILL when this parent dies, however it dies
        import ctypes
        ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGKILL)   # PR_SET_PDEATHSIG

    procs = []

    def forward(signum, frame):   # a launcher's SIGTERM / ^C reaches every rank's process group
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        sys.exit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, forward)
    for cmd, env in rank_commands(argv, gpus, free_port(), os.environ):
        # own session per rank: a failed run kills each rank's whole subtree
        # (its config-5 child too) with one killpg
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True, preexec_fn=die_with_parent))
    rc, failed_at = 0, None
    try:
        while any(p.poll() is None for p in procs):
            for g, p in enumerate(procs):
                if p.returncode not in (None, 0) and rc == 0:
                    rc, failed_at = _exit_status(p.returncode), time.monotonic()
                    print(f"bench.py: rank {g} exited with {p.returncode}", file=sys.stderr, flush=True)
            if failed_at is not None and time.monotonic() - failed_at > grace_s:
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()
    for g, p in enumerate(procs):
        if rc == 0 and p.returncode != 0:
            rc = _exit_status(p.returncode)
            print(f"bench.py: rank {g} exited with {p.returncode}", file=sys.stderr, flush=True)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--batch", type=int, default=0,
                    help="squares per rank per step (default: config 4's 1024 squares split over the ranks, "
                         "1024 // world)")
    ap.add_argument("--distinct", type=int, default=0,
                    help="distinct input squares per rank, tiled to the batch (default: all distinct)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = all host CPUs (capped by OMP_NUM_THREADS)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip k=512 and latency extras")
    ap.add_argument("--config5", action="store_true",
                    help="run the config-5 extra (one k=512 square split over the ranks) even at one rank")
    ap.add_argument("--config5-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--layout", choices=("packed", "inplace"), default="inplace",
                    help="inplace: ODS already in Q0 of the EDS arena (cda_extend_dah_inplace_device, the layout "
                         "rsmt2d's EDS has; no Q0 copy); packed: ODS in its own k*k buffer "
                         "(cda_extend_dah_device, Q0 copied into the EDS)")
    args = ap.parse_args()

    mode = launch_mode(args.gpus, os.environ) if not args.config5_child else "rank"
    if mode == "mismatch":
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE')}: refusing to measure a "
              f"different world size than asked", file=sys.stderr)
        sys.exit(2)
    if mode == "spawn":   # before torch is imported: the parent never touches the GPU
        sys.exit(spawn_ranks(sys.argv[1:], args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cfg5 = None
    if (world > 1 or args.config5) and not args.no_extras and not args.config5_child:
        # config 5: ONE k=512 square split by row blocks over all ranks (RCCL
        # all-to-all of the row-encoded blocks, column encode + hashing per
        # rank, gather of subtree/column roots, combine on rank 0), run by a
        # child process per rank with its own process group: a collective that
        # never returns or a crash there must not cost the headline line.  It
        # runs FIRST, before this rank touches the GPU, so a rank and its child
        # never hold the GPU together: N ranks + N children + a launcher agent
        # would pass a box's 16-processes-per-GPU cap at N = 8
        # (profiles/r06/gpu_procs.txt).
        cfg5 = config5_isolated(world, CONFIG5_TIMEOUT_S)

    import numpy as np
    import torch
    import torch.distributed as dist

    from celestia_da import Context, testfactory
    # rehearsal knobs (never set by the driver): CDA_BENCH_DEVICE puts every
    # rank on one device and CDA_BENCH_BACKEND=gloo replaces RCCL for the
    # parent group, so the N > 1 flow runs on a one-GPU box
    if os.environ.get("CDA_BENCH_DEVICE"):
        local = int(os.environ["CDA_BENCH_DEVICE"])
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or args.config5 or args.config5_child:
        if world == 1:   # a one-rank group for --config5 outside torchrun
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        backend = os.environ.get("CDA_BENCH_BACKEND", "nccl")
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
        assert dist.get_world_size() == world, (dist.get_world_size(), world)
    launch = {"mode": {"rank": "external launcher" if not os.environ.get("CDA_BENCH_LAUNCHER")
                       else "spawned by bench.py --gpus", "inprocess": "single process"}[mode],
              "group_world_size": dist.get_world_size() if dist.is_initialized() else 1,
              "backend": dist.get_backend() if dist.is_initialized() else None}

    if args.config5_child:   # config5_isolated's child: one rank of config 5, JSON on stdout (rank 0)
        def emit(part):
            if rank == 0:
                print("CONFIG5 " + json.dumps(part), flush=True)
        emit(config5(Context(local), dev, rank, world, 512, emit=emit))
        dist.destroy_process_group()
        return

    k = args.k
    # config 4 (BASELINE.json configs[3]): a FIXED workload of 1024 squares
    # split over the ranks -- rank g takes [g*1024/N, (g+1)*1024/N)
    B = args.batch if args.batch > 0 else CONFIG4_SQUARES // world
    W = 2 * k
    ctx = Context(local)

    # inputs: this rank's squares, all distinct unless --distinct asks for
    # tiling; generated on host threads in chunks straight into HBM
    idx = list(shard(rank, world, B))
    nd = B if args.distinct <= 0 else max(1, min(args.distinct, B))
    d_ods = torch.empty((B, k * k, SHARE), dtype=torch.uint8, device=dev)
    t_gen = time.perf_counter()
    for j0, part in testfactory.random_squares(k, idx[:nd]):
        d_ods[j0:j0 + part.shape[0]].copy_(torch.from_numpy(part))
    for j in range(nd, B, nd):   # tiling (timing-diagnostic runs only)
        d_ods[j:j + nd].copy_(d_ods[:min(nd, B - j)])
    t_gen = time.perf_counter() - t_gen
    d_eds = torch.empty(B * W * W * SHARE, dtype=torch.uint8, device=dev)
    d_rows = torch.empty(B * W * 90, dtype=torch.uint8, device=dev)
    d_cols = torch.empty(B * W * 90, dtype=torch.uint8, device=dev)
    d_roots = torch.empty(B * 32, dtype=torch.uint8, device=dev)
    d_status = torch.empty(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step_packed():
        ctx.extend_dah_device(d_ods.data_ptr(), k, B, d_eds.data_ptr(), d_rows.data_ptr(), d_cols.data_ptr(),
                              d_roots.data_ptr(), d_status.data_ptr(), stream)

    def step_inplace():
        ctx.extend_dah_inplace_device(k, B, d_eds.data_ptr(), d_rows.data_ptr(), d_cols.data_ptr(),
                                      d_roots.data_ptr(), d_status.data_ptr(), stream)

    if args.layout == "inplace":
        # the ODS arrives in Q0 of the EDS arena; RS writes only Q1..Q3, so Q0
        # stays intact across steps
        d_eds.view(B, W, W, SHARE)[:, :k, :k] = d_ods.view(B, k, k, SHARE)
        step = step_inplace
    else:
        step = step_packed

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    parity = {"checked": 0, "matched": 0}
    if not os.environ.get("CDA_BENCH_NOCHECK"):   # set only for timing-diagnostic library variants
        assert int(d_status.abs().sum().item()) == 0, "push-order status set on ordered input"
        roots = d_roots.view(B, 32).cpu().numpy()
        if nd < B:   # tiled inputs must give tiled data roots
            for i in range(nd, B):
                assert (roots[i] == roots[i % nd]).all()
        g = golden_config4()
        if g and g.get("k") == k:
            for j, i in enumerate(idx[:nd]):
                want = g["squares"].get(str(i))
                if want is not None:
                    parity["checked"] += 1
                    parity["matched"] += int(roots[j].tobytes().hex() == want["data_root"])
            assert parity["matched"] == parity["checked"], f"data roots differ from the oracle fixture: {parity}"

    def reduce_max(x: float) -> float:
        t = torch.tensor([x], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    if world > 1:   # every rank's shard is checked against the fixture; the line reports all of them
        parity = gather_parity(parity, world, dev if dist.get_backend() == "nccl" else "cpu")

    # the timed region runs the product path exactly as a caller would (no
    # stage events); the per-stage HIP-event breakdown comes from a separate
    # pass afterwards (the events add ~10 us launch gaps at stage borders)
    el = time_region(step, args.steps, lambda: torch.cuda.synchronize(dev), world, reduce_max, dist.barrier)
    ctx.set_profiling(True)
    ctx.stage_times()
    n_prof = max(3, min(args.steps, 10))
    el_prof = time_region(step, n_prof, lambda: torch.cuda.synchronize(dev), 1)
    ctx.set_profiling(False)
    st = ctx.stage_times()

    total_sq = B * world * args.steps
    value = total_sq / el
    stages = stage_report(st, k, B, args.layout == "inplace", n_prof)
    dom = max((s for s in stages if "achieved" in stages[s]), key=lambda s: stages[s]["avg_ms"])
    d = stages[dom]
    traffic = traffic_report(k, B)
    roofline = {"bound": d["bound"], "achieved": d["achieved"], "peak": d["peak"], "unit": d["unit"],
                "frac": d["frac"], "kernel": dom, "launch_ms": d["avg_ms"],
                "work_per_launch": f"{d.get('compressions', 0)} SHA-256 compressions ({B} squares)",
                "frac_issue_slots": d.get("frac_issue_slots"), "frac_of_achievable": d["frac_of_achievable"],
                "traffic": None}
    if dom in traffic:   # per launch like `achieved`: one launch = the stage pass's whole batch
        roofline["traffic"] = traffic[dom]["traffic_per_step"]
        roofline["traffic_ratio"] = traffic[dom]["traffic_ratio"]
    ceiling = combined_ceiling(k)
    roofline["combined_ceiling_squares_per_s"] = ceiling
    roofline["combined_frac"] = (value / world) / ceiling
    rs_ms = sum(stages[s]["avg_ms"] for s in ("rs_q0", "rs_q3") if s in stages)
    rs_alg = rs_bytes(k) * B
    rs_roof = {"bound": "hbm", "achieved": rs_alg / (rs_ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBS,
               "unit": "GB/s", "ms_per_step": rs_ms, "algorithmic_bytes_per_step": rs_alg}
    rs_roof["frac"] = rs_roof["achieved"] / rs_roof["peak"]
    rs_roof["achievable"] = ACHIEVABLE_HBM_GBS
    # measured HBM bytes of the RS launches of one step (PMC summary)
    rs_stage = "rs_gf8_bs" if k == 128 else "rs_gf16"
    if rs_stage in traffic:
        rs_roof["traffic"] = traffic[rs_stage]["traffic_per_step"]
        rs_roof["traffic_ratio"] = traffic[rs_stage]["traffic_ratio"]
    rs_roof["frac_of_achievable"] = rs_roof["achieved"] / ACHIEVABLE_HBM_GBS
    v_rs = load_pmc(rs_stage, "SQ_INSTS_VALU")
    rs_launches = load_pmc(rs_stage, "launches_per_step_k%d" % k) or 2
    v_sq = load_pmc("_config", "k%d" % k) or {}
    if v_rs and v_sq.get("squares_per_step"):
        # per launch of the profiled shape -> per step of this run
        lane = v_rs * rs_launches / v_sq["squares_per_step"] * B * 64 / (rs_ms * 1e-3) / 1e12
        rs_roof["valu"] = {"bound": "valu", "achieved": lane, "peak": PEAK_VALU_TOPS, "unit": "T lane-instr/s",
                           "frac": lane / PEAK_VALU_TOPS, "source": "SQ_INSTS_VALU x 64 per step (PMC summary)"}

    extras = {}
    if rank == 0 and not args.no_extras:
        # config 2: single-square latency at k=128 (one ProcessProposal)
        lat = []
        for _ in range(10):
            torch.cuda.synchronize(dev)
            a = time.perf_counter()
            ctx.extend_dah_device(d_ods.data_ptr(), k, 1, d_eds.data_ptr(), d_rows.data_ptr(), d_cols.data_ptr(),
                                  d_roots.data_ptr(), d_status.data_ptr(), stream)
            torch.cuda.synchronize(dev)
            lat.append(time.perf_counter() - a)
        extras["latency_single_square_ms"] = 1e3 * sorted(lat)[len(lat) // 2]
        # the other device layout, same squares (a few steps, HIP-event stage times)
        other = step_packed if args.layout == "inplace" else step_inplace
        if args.layout == "inplace":
            pass   # packed reads d_ods, still resident
        else:
            d_eds.view(B, W, W, SHARE)[:, :k, :k] = d_ods.view(B, k, k, SHARE)
        other()
        n_o = 5
        el_o = time_region(other, n_o, lambda: torch.cuda.synchronize(dev), 1)
        extras["layout_" + ("packed" if args.layout == "inplace" else "inplace")] = {
            "squares_per_s": n_o * B / el_o, "ms_per_step": 1e3 * el_o / n_o}
        try:
            extras["host_buffers"] = host_buffer_rates(ctx, k)
        except Exception as e:  # report, never lose the headline line
            extras["host_buffers"] = {"error": f"{type(e).__name__}: {e}"}
        try:
            extras["host_buffers_config4"] = host_pipeline_rates(ctx, k, d_ods, d_eds, idx)
        except Exception as e:  # report, never lose the headline line
            extras["host_buffers_config4"] = {"error": f"{type(e).__name__}: {e}"}
        try:
            extras["square_construction"] = square_construction(ctx, dev, stream)
        except Exception as e:  # report, never lose the headline line
            extras["square_construction"] = {"error": f"{type(e).__name__}: {e}"}
        try:
            extras["blob_commitments"] = blob_commitments(ctx, dev, stream)
        except Exception as e:
            extras["blob_commitments"] = {"error": f"{type(e).__name__}: {e}"}
        try:
            extras["share_proofs"] = share_proofs(ctx)
        except Exception as e:
            extras["share_proofs"] = {"error": f"{type(e).__name__}: {e}"}
        try:
            extras["eds_repair"] = eds_repair(ctx)
        except Exception as e:
            extras["eds_repair"] = {"error": f"{type(e).__name__}: {e}"}
        # config 3: one 512 x 512 square (GF(2^16), 512 MiB EDS)
        del d_eds
        torch.cuda.empty_cache()
        k5 = 512
        o5 = torch.from_numpy(testfactory.random_square(k5, 0)).to(dev)
        e5 = torch.empty(4 * k5 * k5 * SHARE, dtype=torch.uint8, device=dev)
        r5 = torch.empty(2 * k5 * 90, dtype=torch.uint8, device=dev)
        c5 = torch.empty(2 * k5 * 90, dtype=torch.uint8, device=dev)
        g5 = torch.empty(32, dtype=torch.uint8, device=dev)

        # in place, like the headline (the ODS already in Q0 of the EDS arena,
        # the layout rsmt2d's EDS has); the packed entry timed beside it
        e5.view(2 * k5, 2 * k5, SHARE)[:k5, :k5] = o5.view(k5, k5, SHARE)

        def step5():
            ctx.extend_dah_inplace_device(k5, 1, e5.data_ptr(), r5.data_ptr(), c5.data_ptr(), g5.data_ptr(), None,
                                          stream)
        # Warm-up: back-to-back one-square steps speed up over their first
        # ~30 calls (1.08-1.20 -> 0.98 ms per step in a kernel trace,
        # profiles/r05/k512_step_trace.txt), so 5 steps right after 12
        # warm-up calls (the round-4 timing, kept as "first_steps") sit on the
        # ramp; the steady-state figure times 20 steps after 40.
        for _ in range(12):
            step5()
        torch.cuda.synchronize(dev)
        n5 = 5
        a = time.perf_counter()
        for _ in range(n5):
            step5()
        torch.cuda.synchronize(dev)
        el5c = time.perf_counter() - a
        for _ in range(23):
            step5()
        torch.cuda.synchronize(dev)
        n5s = 20
        # event-free timing (as the headline); the stage breakdown from a
        # separate profiled pass (its events add launch gaps at stage borders)
        a = time.perf_counter()
        for _ in range(n5s):
            step5()
        torch.cuda.synchronize(dev)
        el5 = (time.perf_counter() - a) * n5 / n5s   # per n5 squares, like the passes below
        ctx.set_profiling(True)
        ctx.stage_times()
        a = time.perf_counter()
        for _ in range(n5):
            step5()
        torch.cuda.synchronize(dev)
        el5p = time.perf_counter() - a
        ctx.set_profiling(False)
        # per step: the levels stage is marked twice per step (wide levels, tree top)
        st5 = stage_report(ctx.stage_times(), k5, 1, True, n5)

        def step5p():
            ctx.extend_dah_device(o5.data_ptr(), k5, 1, e5.data_ptr(), r5.data_ptr(), c5.data_ptr(), g5.data_ptr(),
                                  None, stream)
        step5p()
        torch.cuda.synchronize(dev)
        a = time.perf_counter()
        for _ in range(n5):
            step5p()
        torch.cuda.synchronize(dev)
        el5k = time.perf_counter() - a
        extras["k512"] = {"squares_per_s": n5 / el5, "ms_per_square": 1e3 * el5 / n5,
                          "layout": "inplace", "timing": "20 steps after 40 warm-up calls",
                          "first_steps": {"ms_per_square": 1e3 * el5c / n5,
                                          "timing": "5 steps after 12 warm-up calls (on the warm-up ramp)"},
                          "ms_per_square_profiled_pass": 1e3 * el5p / n5,
                          "packed": {"squares_per_s": n5 / el5k, "ms_per_square": 1e3 * el5k / n5},
                          "ods_gb_per_s": n5 * k5 * k5 * SHARE / el5 / 1e9,
                          "data_root": g5.cpu().numpy().tobytes().hex(),
                          "combined_ceiling_squares_per_s": combined_ceiling(k5),
                          "combined_frac": (n5 / el5) / combined_ceiling(k5),
                          "stages": st5}
        gk = golden_k512()
        if gk:
            extras["k512"]["data_root_matches_oracle"] = extras["k512"]["data_root"] == gk["0"]["data_root"]
        rs5 = sum(st5[s]["avg_ms"] for s in ("rs_q0", "rs_q3") if s in st5)
        extras["k512"]["rs_roofline"] = {"bound": "hbm", "ms_per_square": rs5,
                                         "achieved": rs_bytes(k5) / (rs5 * 1e-3) / 1e9, "peak": PEAK_HBM_GBS,
                                         "unit": "GB/s", "frac": rs_bytes(k5) / (rs5 * 1e-3) / 1e9 / PEAK_HBM_GBS}
        v16 = load_pmc("rs_gf16", "SQ_INSTS_VALU")   # per launch of the profiled k=512 run
        n16 = load_pmc("rs_gf16", "launches_per_step_k512") or 2
        c16 = (load_pmc("_config", "k512") or {}).get("squares_per_step") or 1
        t16 = traffic_report(k5, 1)
        if t16:
            extras["k512"]["traffic"] = t16
        if v16:
            lane = v16 * n16 / c16 * 64 / (rs5 * 1e-3) / 1e12
            clk = load_pmc("rs_gf16", "effective_clock_ghz") or 2.4
            # The bitsliced encoder (round 4) is an all-full-rate stream (v_bitop3 /
            # v_xor networks; tests/test_bitslice16.py asserts it): a SIMD-32
            # issues one wave64 instruction per 2 cycles, so the ceiling is
            # 1024 SIMDs x 64 lanes / 2 x the measured clock (the round-3
            # half-rate v_perm model no longer applies).
            issue = 1024 * 64 / 2 * clk * 1e9 / 1e12
            extras["k512"]["rs_roofline"]["valu"] = {
                "achieved": lane, "peak": PEAK_VALU_TOPS, "unit": "T lane-instr/s", "frac": lane / PEAK_VALU_TOPS,
                "full_rate_issue_ceiling": issue, "frac_of_issue_ceiling": lane / issue, "clock_ghz": clk,
                "source": "SQ_INSTS_VALU x 64 per square (PMC summary, one-square run), clock GRBM_GUI_ACTIVE; "
                          "ceiling = 1024 x 64 / 2 x clock (full-rate issue)"}
        # the same square 2 and 4 times per submission: the latency-bound tail
        # (top NMT levels, 12-level data-root chain) is shared by the squares
        del e5
        torch.cuda.empty_cache()
        for nb in (2, 4):
            ob = o5.repeat(nb, 1)
            eb = torch.empty(nb * 4 * k5 * k5 * SHARE, dtype=torch.uint8, device=dev)
            rb = torch.empty(nb * 2 * k5 * 90, dtype=torch.uint8, device=dev)
            cb = torch.empty(nb * 2 * k5 * 90, dtype=torch.uint8, device=dev)
            gb = torch.empty(nb * 32, dtype=torch.uint8, device=dev)

            eb.view(nb, 2 * k5, 2 * k5, SHARE)[:, :k5, :k5] = ob.view(nb, k5, k5, SHARE)   # in place, as above

            def stepb():
                ctx.extend_dah_inplace_device(k5, nb, eb.data_ptr(), rb.data_ptr(), cb.data_ptr(), gb.data_ptr(), None,
                                              stream)
            stepb()
            torch.cuda.synchronize(dev)
            a = time.perf_counter()
            for _ in range(n5):
                stepb()
            torch.cuda.synchronize(dev)
            elb = time.perf_counter() - a
            assert bytes(gb.view(nb, 32)[nb - 1].cpu().numpy()) == bytes(g5.cpu().numpy()), "k512 batch data root"
            extras["k512"][f"batch{nb}"] = {"squares_per_s": n5 * nb / elb, "ms_per_square": 1e3 * elb / (n5 * nb)}
            del ob, eb
            torch.cuda.empty_cache()

    def make_line(cpu):
        return {
            "metric": "EDS+DAH squares/sec (k=128)",
            "value": value,
            "unit": "squares/s",
            "n_gpus": world,
            "launch": launch,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * el / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if B * world == CONFIG4_SQUARES else "weak",
            "vs_baseline": None,
            "dtype": "u8/u32",
            "data": (f"synthetic random-namespace squares (testfactory mirror, SplitMix64), "
                     f"{'all distinct' if nd == B else f'{nd} distinct tiled'}: square indexes "
                     f"{idx[0]}..{idx[-1]} on rank 0 (generated on host threads in {t_gen:.1f} s, "
                     f"HBM-resident before timing)"),
            "config": {"workload": (f"config 4: {B * world} independent k={k} squares per step split over "
                                    f"{world} GPU(s), {B} per GPU (rank g: squares [{B}g, {B}g+{B}))"
                                    if B * world == CONFIG4_SQUARES else
                                    f"{B} independent k={k} squares per GPU per step (not config 4's fixed "
                                    f"1024-square workload)"),
                       "k": k, "squares_per_step": B * world, "squares_per_gpu_per_step": B,
                       "distinct_squares": nd, "parallelism": f"dp{world} (independent squares)",
                       "layout": args.layout},
            "parity": {**parity, "fixture": "tests/golden/config4_k128{,_rest}.json (oracle data roots of squares 0..1023)"},
            "ods_gb_per_s": value * k * k * SHARE / 1e9,
            "stage_pass": {"steps": n_prof, "ms_per_step": 1e3 * el_prof / n_prof,
                           "note": "stages and rooflines come from this separate pass with HIP events at every "
                                   "stage border, on the one-stream schedule; value / ms_per_step come from the "
                                   "event-free timed region, whose hash stages run on " +
                                   ("two streams (enqueue_dah splits batches of < 64 squares at k <= 128)"
                                    if B < 64 and k <= 128 else
                                    "one stream (enqueue_dah splits only batches of < 64 squares at k <= 128)")},
            "roofline": roofline,
            "rs_roofline": rs_roof,
            "traffic": traffic,
            "stages": stages,
            "cpu_baseline": cpu,
            "extras": extras,
        }

    if cfg5 is not None:   # measured first, see above
        extras["config5"] = cfg5

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:   # the CPU baseline is an N=1 figure
        cpu = cpu_baseline(k, args.cpu_seconds, args.cpu_threads)

    if rank == 0:
        print(json.dumps(make_line(cpu)))
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
