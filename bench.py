#!/usr/bin/env python3
"""Benchmark: device-resident SSTable decode (BASELINE.json config 2).

One step = one hg_decode_dev_async over a 1 GiB SSTable already in HBM
(8,134,407 records of 16 B big-endian counter keys / 100 B random values,
seed 2, built on the device): boundary discovery + one span per record.
With --gpus N (launched by torch.distributed.run) every rank decodes its own
table on its own GPU: weak scaling, no collectives on the data path (the only
collectives are the timing barrier and the max-over-ranks reduction).

Prints ONE JSON line (rank 0).  `roofline` prices one decode call against
HBM: algorithmic bytes = L + 16 n (read the table once, write 16-byte spans),
divided by the call's duration measured with HIP events on the stream its
kernels run on.  A decode call is a short pipeline (decode_spec_kernel,
decode_kernel -- the latter writes the spans of the pre-pass's resolved
prefix and runs the general engine on the rest; the statuses are cleared by
the previous call's pre-pass, so repeated calls launch no memset); the
stride pre-pass dominates (profiles/).  `cpu_baseline` times the oracle
(the C restatement of the reference's Rust decode, with its per-record
ownership pattern) on one host core over the same bytes.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
CFG2 = dict(n=8_134_407, k=16, v=100, seed=2)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse(argv=None):
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--cpu-sample-mb", type=int, default=1024,
                   help="bytes of the same table the CPU baseline decodes per pass (0 = skip)")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="repeat CPU baseline passes until this much CPU time is spent")
    p.add_argument("--no-encode", action="store_true", help="skip the config-3 encode leg")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the config-4 / config-5 (scaled) legs")
    p.add_argument("--no-host", action="store_true",
                   help="skip the host-inclusive (H2D + kernel + D2H) legs")
    p.add_argument("--multi-split-child", default=None, metavar="DEVICES",
                   help=argparse.SUPPRESS)  # internal: the cross-GPU leg's own process
    return p.parse_args(argv)


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def shard_plan(rank, world):
    """Weak scaling: every rank decodes its own full cfg2 table (independent
    tables, no data-path exchange); only the seed differs per rank."""
    return dict(CFG2, seed=CFG2["seed"] + 1000 * rank, rank=rank, world=world)


def aggregate(wall_max_s, steps, world, bytes_per_rank):
    """Whole-job rate: the bytes all ranks decoded / the slowest rank's time."""
    return world * bytes_per_rank / (wall_max_s / steps) / GIB


def _backend():
    return os.environ.get("HG_BENCH_DIST_BACKEND", "nccl")


def max_over_ranks(value, world, device=None):
    """Max of a float across ranks (identity when world == 1)."""
    if world == 1:
        return value
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64,
                     device=None if _backend() == "gloo" else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


_SIDE = None  # a gloo group over all ranks: CPU-side waits (no kernel on the GPUs)


def init_side_group():
    """Every rank calls this once after init_process_group."""
    global _SIDE
    import torch.distributed as dist
    _SIDE = dist.new_group(backend="gloo")


def side_barrier(world):
    """Barrier on the gloo side group: a rank waiting here runs nothing on
    its GPU -- an RCCL barrier would keep an allreduce kernel spinning on the
    GPUs rank 0 drives in the cross-GPU leg."""
    if world > 1:
        import torch.distributed as dist
        dist.barrier(group=_SIDE)


def barrier(world, device=None):
    if world > 1:
        import torch.distributed as dist
        if device is not None and device.type == "cuda" and _backend() != "gloo":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


DECODE_KERNELS = ("decode_spec_kernel", "decode_kernel")
PMC_TAG = "r6"  # the round whose profiles/<tag>_pmc_*.json the legs cite


def load_traffic(kernels):
    """(HBM bytes per decode call summed over its kernels, source commit of
    the PMC summary) from the committed profiles/pmc_summary.json; (None,
    None) if it does not cover every kernel."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path, encoding="utf-8") as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None, None
    vals = [pmc.get(k, {}).get("hbm_bytes_per_launch") for k in kernels]
    src = dict(pmc.get("_source", {}))
    try:  # does the summary describe the decode kernels being run now?
        import hashlib
        cur = hashlib.sha256(open(os.path.join(ROOT, "horreum_amd", "csrc", "hg_decode.hip"),
                                  "rb").read()).hexdigest()
        src["current_source"] = src.get("hg_decode_sha256") == cur
    except OSError:
        src["current_source"] = None
    return (None if any(v is None for v in vals) else float(sum(vals))), src


def time_async(torch, fn, steps, warmup, world, device):
    """Run fn() warmup+steps times; returns (wall_s_max_over_ranks, per-launch
    ms list).  The launch time is the HIP-event time of the whole timed loop
    on its stream divided by `steps` (one event pair brackets the loop:
    events between the steps cost ~10 us each on the cfg 2 headline,
    tools/event_overhead.py), so it includes the gaps between launches."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(device)
    stream = torch.cuda.current_stream(device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world, device)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        fn()
    ev1.record(stream)
    torch.cuda.synchronize(device)
    barrier(world, device)
    wall = time.perf_counter() - t0
    launch_ms = [ev0.elapsed_time(ev1) / steps] * steps
    return max_over_ranks(wall, world, device), launch_ms


def cpu_baseline(sst_dev, n_records, sample_mb, seconds):
    """Oracle (C restatement of src/format.rs:50-77, owned buffers) on 1 core:
    decode passes over (a prefix of) the same table until `seconds` of CPU
    decode time have been spent."""
    if sample_mb <= 0:
        return None
    from oracle import oracle
    rec = 16 + CFG2["k"] + CFG2["v"]
    nrec = min(n_records, (sample_mb << 20) // rec)
    host = sst_dev[: nrec * rec].cpu().numpy()
    total_s, passes = 0.0, 0
    while passes == 0 or total_s < seconds:
        n, secs = oracle.bench_decode_owned(host)
        assert n == nrec, (n, nrec)
        total_s += secs
        passes += 1
    return {"value": round(passes * host.size / total_s / GIB, 4), "unit": "GiB/s", "cores": 1,
            "kind": "port",
            "sample": f"{passes} passes over the first {nrec} records ({host.size} B) of the "
                      f"same table, hgo_bench_decode_owned, {total_s:.2f} s",
            "all_cores": cpu_all_cores(host),
            "extra": cpu_extras(host)}


def host_cores():
    """(threads to use, the machine's nproc, this process's CPU affinity): the
    GPU box gives one GPU's job a share of a larger machine (OMP_NUM_THREADS
    holds that share), so nproc alone overstates it."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff
    return max(1, min(share, aff)), nproc, aff


def cpu_all_cores(host_sample, seconds=1.0):
    """The optimised multi-threaded CPU codec (oracle/cpu_opt.c: byte ranges
    with guessed entries handed over in order, spans placed in parallel, not
    owned copies; sizes / prefix / copy for encode; workers started at a
    barrier, as a pool would hold them) at several thread counts up to EVERY
    core this process may run on (its CPU affinity, capped at the codec's 256
    threads), the job's OMP_NUM_THREADS share among them: cfg 2 decode of the
    same sample, cfg 3 encode of a 1 M-pair sample, and a memcpy of the
    sample (the CPU's streaming ceiling); the best of each is the figure."""
    from horreum_amd import synth
    from oracle import oracle
    share, nproc, aff = host_cores()
    want_n = host_sample.size // (16 + CFG2["k"] + CFG2["v"])
    arena, pairs = synth.fixed_arena(1_000_000, 32, 256, seed=3, device="cpu")
    a, p = arena.numpy(), pairs.numpy().view(oracle.PAIR_DTYPE)
    out = np.empty(304_000_000, dtype=np.uint8)
    cp = np.empty_like(host_sample)
    spans = np.zeros(host_sample.size // 16 + 1, dtype=oracle.SPAN_DTYPE)

    def rate(fn, nbytes):
        tot, k = 0.0, 0
        while k == 0 or tot < seconds:
            tot += fn()
            k += 1
        return k * nbytes / tot / GIB

    def measure(threads):
        scratch = np.empty(host_sample.size // 16 + 2 * threads + 2, dtype=oracle.SPAN_DTYPE)

        def dec():
            _, n, t = oracle.mt_decode(host_sample, threads, spans, scratch)
            assert n == want_n, (n, want_n)
            return t

        def enc():
            got, t = oracle.mt_encode(a, p, threads, out)
            assert got.size == 304_000_000
            return t
        return {"threads": threads,
                "decode_cfg2_GiB_s": round(rate(dec, host_sample.size), 3),
                "encode_cfg3_1M_GiB_s": round(rate(enc, 304_000_000), 3),
                "memcpy_GiB_s": round(rate(lambda: oracle.mt_memcpy(cp, host_sample, threads),
                                           host_sample.size), 3)}
    # thread counts: the job's share, powers of two up to every core of the
    # affinity (the memory system, not the core count, bounds this byte work:
    # more threads are not always faster), the codec's 256-thread cap
    counts = sorted({c for c in (share, 32, 64, 128, min(aff, 256)) if 1 <= c <= min(aff, 256)})
    runs = [measure(c) for c in counts]
    ok = bool(np.array_equal(spans[:1000], oracle.decode(host_sample[:132000])[0])
              and np.array_equal(cp[:4096], host_sample[:4096]))
    del cp
    best = max(runs, key=lambda r: r["decode_cfg2_GiB_s"])
    return {"cores": best["threads"], "nproc": nproc, "affinity": aff, "kind": "port (tuned)",
            "decode_cfg2_GiB_s": best["decode_cfg2_GiB_s"],
            "encode_cfg3_1M_GiB_s": max(r["encode_cfg3_1M_GiB_s"] for r in runs),
            "memcpy_GiB_s": max(r["memcpy_GiB_s"] for r in runs),
            "by_threads": runs,
            "sample": f"decode: the same {host_sample.size} B cfg 2 sample; encode: 1 M pairs of "
                      f"32 B / 256 B; hgo_mt_decode / hgo_mt_encode, >= {seconds} s each, at "
                      f"{counts} threads (every core of the process's affinity the largest); the "
                      f"best of each is reported",
            "parity_spot": ok}


def cpu_extras(host_sample, seconds=1.0):
    """The rest of BASELINE.md's CPU plan, on the same host core: cfg 1 (the
    reference's own CPU case: 100 k puts of 16 B keys / 100 B values ->
    serialize_flatten -> full iteration with deserialize_from_bytes, owned
    buffers as src/format.rs:23-77), the cfg 3 owned encode on a 1 M-pair
    sample, the oracle's allocation-free span decode (a tuned single-thread
    decode: the serial walk cannot be split across cores without the
    speculation the GPU does) and a single-thread host memcpy of the sample
    (the CPU's own streaming ceiling for this byte work)."""
    from horreum_amd import synth
    from oracle import oracle

    def rep(fn):
        tot, k = 0.0, 0
        while k == 0 or tot < seconds:
            tot += fn()
            k += 1
        return tot / k

    out = {"cores": 1}
    arena, pairs = synth.fixed_arena(100_000, 16, 100, seed=1, device="cpu")
    a, p = arena.numpy(), pairs.numpy().view(oracle.PAIR_DTYPE)
    table, _, _, _ = oracle.encode(a, p)
    te = rep(lambda: oracle.bench_encode_owned(a, p)[1])
    td = rep(lambda: oracle.bench_decode_owned(table)[1])
    out["cfg1_100k_puts"] = {"bytes": int(table.size), "encode_ms": round(te * 1e3, 3),
                             "iterate_ms": round(td * 1e3, 3),
                             "encode_GiB_s": round(table.size / te / GIB, 4),
                             "iterate_GiB_s": round(table.size / td / GIB, 4)}
    arena, pairs = synth.fixed_arena(1_000_000, 32, 256, seed=3, device="cpu")
    a, p = arena.numpy(), pairs.numpy().view(oracle.PAIR_DTYPE)
    te = rep(lambda: oracle.bench_encode_owned(a, p)[1])
    out["cfg3_encode_owned_1M"] = {"bytes": 304_000_000, "GiB_s": round(304e6 / te / GIB, 4)}

    def span_decode():
        t0 = time.perf_counter()
        oracle.decode(host_sample)
        return time.perf_counter() - t0

    td = rep(span_decode)
    out["cfg2_span_decode_tuned"] = {"bytes": int(host_sample.size),
                                     "GiB_s": round(host_sample.size / td / GIB, 4)}
    dst = np.empty_like(host_sample)

    def cp():
        t0 = time.perf_counter()
        np.copyto(dst, host_sample)
        return time.perf_counter() - t0

    tc = rep(cp)
    out["host_memcpy_GiB_s"] = round(host_sample.size / tc / GIB, 3)
    return out


_T0 = time.time()


def progress(rank, what):
    """One stderr line per finished leg (stdout carries only the JSON line):
    a long run -- the N > 1 rehearsals share one card -- shows it is alive."""
    print(f"[bench rank {rank}] {what} done at {time.time() - _T0:.1f} s", file=sys.stderr, flush=True)


def multi_split_isolated(devices, timeout_s=600):
    """multi_split_leg in a child process (rank 0 waits on it): the leg drives
    every GPU of the node from one process, through the peer-copy branch, and
    a fault there must not cost the bench line the driver's N > 1 runs
    record.  Returns the child's JSON object, or an error record."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--multi-split-child",
           ",".join(str(d) for d in devices)]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                        "ROLE_RANK", "TORCHELASTIC_RUN_ID")}
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, env=env)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {timeout_s} s"}
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"exit {p.returncode}", "stderr_tail": p.stderr[-600:]}
    out = json.loads(lines[-1])
    out["process"] = "child of rank 0 (isolated from the bench line)"
    return out


def multi_split_child(devs):
    import torch
    from horreum_amd.engine import Engine
    devices = [int(x) for x in devs.split(",")]
    torch.cuda.set_device(devices[0])
    eng = Engine(devices[0])
    try:
        out = multi_split_leg(torch, eng, devices)
    except Exception as e:  # noqa: BLE001 -- reported, not raised
        out = {"error": repr(e)}
    print(json.dumps(out), flush=True)
    return 0


def main(argv=None):
    args = parse(argv)
    if args.multi_split_child:
        return multi_split_child(args.multi_split_child)
    rank, world, local = dist_env()
    import torch
    if os.environ.get("HG_BENCH_SHARE_GPU") == "1":
        # rehearsal of the N > 1 path on a one-GPU box (ranks share the card,
        # gloo for the timing collectives); the driver's runs never set it
        local = local % max(1, torch.cuda.device_count())
        os.environ["HG_BENCH_DIST_BACKEND"] = "gloo"
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if _backend() == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        init_side_group()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    from horreum_amd import synth
    from horreum_amd.engine import Engine

    eng = Engine(local)
    plan = shard_plan(rank, world)
    n, k, v = plan["n"], plan["k"], plan["v"]
    sst = synth.fixed_sst(n, k, v, seed=plan["seed"], device=device)
    L = sst.numel()
    eng.reserve(L, 0)
    spans = eng.empty(n * 16)
    res = eng.empty(64)

    def step():
        eng.decode_dev_async(sst, L, spans, n, res)

    wall, launch_ms = time_async(torch, step, args.steps, args.warmup, world, device)
    progress(rank, "headline decode")

    # correctness of what was timed (outside the timed region)
    r = res[:24].cpu().numpy()
    nrec = int(r[:8].view("<u8")[0])
    kind = int(r[8:12].view("<i4")[0])
    sp = spans[: n * 16].view(torch.int64).view(n, 2)
    idx = torch.arange(n, device=device, dtype=torch.int64)
    ok = (nrec == n and kind == 0 and torch.equal(sp[:, 0], idx * (16 + k + v))
          and bool((sp[:, 1] == (k | (v << 32))).all()))

    ms_step = wall / args.steps * 1e3
    value = aggregate(wall, args.steps, world, L)
    mean_launch_ms = sum(launch_ms) / len(launch_ms)
    alg_bytes = L + 16 * n
    achieved = alg_bytes / (mean_launch_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(DECODE_KERNELS)

    extra = {}
    if not args.no_encode:
        extra["encode_cfg3"] = encode_leg(torch, eng, device, args, world, rank)
        progress(rank, "encode")
    if not args.no_extra:
        del spans
        torch.cuda.empty_cache()
        extra["multi_table_decode_cfg4"] = multi_table_leg(torch, eng, device, args, world, rank,
                                                           host=not args.no_host and world == 1)
        progress(rank, "cfg 4 batched decode")
        extra["compaction_cfg5_scaled"] = compaction_leg(torch, eng, device, world, rank,
                                                         host=not args.no_host and world == 1,
                                                         exact=True)
        progress(rank, "compaction (scaled)")
        extra["compaction_cfg5_share"] = compaction_leg(torch, eng, device, world, rank,
                                                        per_table=8_134_407, exact=True,
                                                        pmc_name=f"{PMC_TAG}_pmc_compaction_share.json",
                                                        host=not args.no_host and world == 1,
                                                        pinned=True)
        progress(rank, "compaction (share)")

    if not args.no_extra:
        extra["decode_general"] = general_legs(torch, eng, device, world)
        extra["lookups"] = lookup_leg(torch, eng, sst, n, k, v)
        progress(rank, "general shapes + lookups")
    if not args.no_host and world == 1:
        extra["host_inclusive"] = host_leg(torch, eng, sst, n, world)
        progress(rank, "host-inclusive")

    if not args.no_extra:
        # the split across GPUs (§8e) from rank 0 over contexts on devices
        # 0..N-1 while the other ranks wait; on one GPU, HG_BENCH_MULTI_CTX=G
        # rehearses it with G contexts sharing the card
        ctx_env = int(os.environ.get("HG_BENCH_MULTI_CTX", "0"))
        ndev = torch.cuda.device_count()
        devices = (list(range(world)) if world > 1 and ndev >= world and
                   os.environ.get("HG_BENCH_SHARE_GPU") != "1" else
                   [local] * ctx_env if ctx_env > 1 else None)
        # the other ranks wait on the gloo side group: nothing of theirs runs
        # on the GPUs rank 0 drives meanwhile
        torch.cuda.synchronize(device)
        side_barrier(world)
        if devices is None:
            extra["multi_gpu_split"] = {"skipped": "one GPU and HG_BENCH_MULTI_CTX unset"}
        elif rank == 0:
            extra["multi_gpu_split"] = multi_split_isolated(devices)
            progress(rank, "cross-GPU split")
        side_barrier(world)

    cpu = (cpu_baseline(sst, n, args.cpu_sample_mb, args.cpu_seconds)
           if (rank == 0 and world == 1) else None)
    if cpu is not None:
        progress(rank, "CPU baseline")
    if rank == 0:
        line = {
            "metric": "GiB/s SSTable bytes encoded+decoded, device-resident, 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device Philox, seed 2 + 1000*rank)",
            "value_is": "decode of BASELINE configs[1] (cfg2), GiB/s of SSTable bytes; encode "
                        "(cfg3) and the other configs are under extra",
            "config": {"workload": "cfg2 single-SSTable decode (BASELINE configs[1])",
                       "records_per_gpu": n, "sst_bytes_per_gpu": L, "key_bytes": k,
                       "value_bytes": v, "decode_piece_bytes": 16384,
                       "prepass_batch_pieces": "adaptive: ~4 workgroups per CU, 64 at cfg2",
                       "parallelism": f"table-per-gpu x{world}, no collectives"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": "decode call: decode_spec_kernel (dominant) + "
                                   "decode_kernel (prefix spans + general engine)",
                         "alg_bytes_per_launch": alg_bytes,
                         "mean_launch_ms": round(mean_launch_ms, 5)},
            "cpu_baseline": cpu,
            "parity": {"spans_checked": bool(ok), "n_records": nrec, "kind": kind},
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0 if ok else 1


GENERAL_SHAPES = [  # (key, label, records, key range, value range, tombstones, seed, zero values)
    ("small", "small mixed 0..24B/0..64B", 4_000_000, (0, 24), (0, 64), 0.05, 4, False),
    ("medium", "medium 8..64B/64..512B", 1_500_000, (8, 65), (64, 513), 0.05, 4, False),
    ("midlarge", "midlarge 16B/400..1200B", 1_000_000, (16, 17), (400, 1201), 0.05, 4, False),
    ("zmidlarge", "zero-valued midlarge 16B/400..1200B", 1_000_000, (16, 17), (400, 1201), 0.0, 9,
     True),
    ("zsmall", "zero-valued small 1..23B/0..63B", 3_000_000, (1, 24), (0, 64), 0.0, 9, True),
]


def load_leg_pmc(name, sources):
    """A bench leg's PMC summary (tools/summarize_pmc.py): per-kernel HBM
    bytes and the sha256 of the sources it was taken at; current_source says
    whether those are the sources being run now."""
    import hashlib
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path, encoding="utf-8") as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return {}, {"file": None}
    src = dict(pmc.get("_source", {}))
    cur = {}
    for s in sources:
        try:
            cur[s] = hashlib.sha256(open(os.path.join(ROOT, "horreum_amd", "csrc", s), "rb").read()).hexdigest()
        except OSError:
            cur[s] = None
    src["file"] = f"profiles/{name}"
    src["current_source"] = all(src.get("sha256", {}).get(s) == h for s, h in cur.items())
    src.pop("sha256", None)
    return pmc.get("kernels", {}), src


def general_legs(torch, eng, device, world, reps=8):
    """Decode of variable-size records (no stride run): small (0-24 B keys /
    0-64 B values) and medium (8-64 B / 64-512 B) records -- the lane-walk
    pre-pass --, 400-1200 B records (hop mode), and the same mid-size and
    small shapes with all-zero value bytes (every 16 value bytes read as an
    empty record: the guesses' worst case).  Device resident; roofline
    against the headline's algorithmic bytes (L + 16 n), HIP-event time of
    the decode call; every span checked against the generator's own record
    layout; PMC traffic from the committed, source-hashed profile of the
    shape (profiles/<PMC_TAG>_pmc_<shape>.json)."""
    from horreum_amd import synth
    out = {}
    for key, label, m, kr, vr, tomb, seed, zero in GENERAL_SHAPES:
        host, g_off, g_kl, g_vl = synth.mixed_sst_host(m, kr, vr, tomb, seed, layout=True,
                                                       zero_values=zero)
        sst = torch.from_numpy(host).to(device)
        L = host.size
        cap = L // 16
        spans = eng.empty(cap * 16)
        res = eng.empty(64)
        eng.reserve(L, 0)

        def step():
            eng.decode_dev_async(sst, L, spans, cap, res)

        wall, ms = time_async(torch, step, reps, 2, world, device)
        mean_ms = sum(ms) / len(ms)
        want = synth.span_rows(g_off, g_kl, g_vl)
        wn = m
        nn = int(res[:8].cpu().numpy().view("<u8")[0])
        kind = int(res[8:12].cpu().numpy().view("<i4")[0])
        ok = nn == wn and kind == 0 and bool(np.array_equal(
            spans[: nn * 16].cpu().numpy().view("<u8").reshape(-1, 2), want))
        alg = L + 16 * wn
        kern, src = load_leg_pmc(f"{PMC_TAG}_pmc_{key}.json", ("hg_decode.hip",))
        traffic = sum(v.get("hbm_read_bytes", 0) + v.get("hbm_write_bytes", 0)
                      for k, v in kern.items() if "decode" in k) or None
        out[key] = {"workload": label, "bytes": L, "records": wn,
                    "ms": round(mean_ms, 4), "value_GiB_s": round(L / (mean_ms * 1e-3) / GIB, 2),
                    "roofline": {"bound": "hbm", "achieved": round(alg / (mean_ms * 1e-3) / 1e9, 1),
                                 "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(alg / (mean_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                 "traffic": traffic, "traffic_source": src},
                    "parity_ok": ok}
        del sst, spans
        torch.cuda.empty_cache()
    return out


def lookup_leg(torch, eng, sst, n, k, v, batch=1 << 20):
    """SSTable::get (src/sstable/table.rs:54-70) for 1 M-key batches against
    the cfg 2 table resident in HBM (spans + key index built once): lookups
    per second, half the keys present, half absent."""
    from horreum_amd import synth
    L = sst.numel()
    out = eng.decode_dev(sst, L)
    idx = eng.keyindex_build(sst, out.spans, out.n)
    g = torch.Generator(device=sst.device)
    g.manual_seed(7)
    ids = torch.randint(0, 2 * n, (batch,), device=sst.device, generator=g)
    keys = synth.be_counter_keys(2 * n, k, sst.device)[ids].contiguous()  # [batch, k]
    q = torch.empty((batch, 2), dtype=torch.int64, device=sst.device)
    q[:, 0] = torch.arange(batch, device=sst.device) * k
    q[:, 1] = k
    res = eng.empty(batch * 24)

    def step():
        eng.lookup_dev_async(sst, out.spans, idx, out.n, keys.view(-1), q.view(torch.uint8),
                             batch, res, 10)

    wall, ms = time_async(torch, step, 10, 2, 1, sst.device)
    r = res.cpu().numpy().view(np.dtype([("rec", "<u8"), ("val_off", "<u8"), ("vlen", "<u4"),
                                         ("found", "<i4")]))
    ids_h = ids.cpu().numpy()
    ok = bool(np.array_equal(r["found"] != 0, ids_h < n)
              and np.array_equal(r["rec"][ids_h < n], ids_h[ids_h < n]))
    mean_ms = sum(ms) / len(ms)
    del idx, keys, q, res
    torch.cuda.empty_cache()
    return {"lookups_per_s": round(batch / (mean_ms * 1e-3)), "batch": batch,
            "ms_per_batch": round(mean_ms, 4), "table": "cfg2 (8.1 M records, resident, blocks of 10)",
            "parity_ok": ok}


def encode_leg(torch, eng, device, args, world, rank):
    """BASELINE config 3: 10 M pairs (32 B / 256 B) -> 3.04 GB of SSTable bytes."""
    from horreum_amd import synth
    n, k, v = 10_000_000, 32, 256
    arena, pairs = synth.fixed_arena(n, k, v, seed=3 + 1000 * rank, device=device)
    total = n * (16 + k + v)
    out = eng.empty(total)
    res = eng.empty(64)
    eng.reserve(0, n)

    def step():
        eng.encode_dev_async(arena, pairs, n, out, total, None, 0, None, res)

    steps = max(1, args.steps // 2)
    wall, launch_ms = time_async(torch, step, steps, max(1, args.warmup // 2), world, device)
    r = res[:16].cpu().numpy()
    out_len = int(r[:8].view("<u8")[0])
    rr = out.view(n, 16 + k + v)
    hdr = torch.zeros(16, dtype=torch.uint8, device=device)
    hdr[0], hdr[8], hdr[9] = k, v & 0xFF, v >> 8  # [u64 LE klen][u64 LE vlen] (src/format.rs:24-28)
    ok = (out_len == total and torch.equal(rr[:, 16:], arena.view(n, k + v))
          and bool((rr[:, :16] == hdr).all()))
    mean_ms = sum(launch_ms) / len(launch_ms)
    alg = n * (k + v) + 24 * n + total  # read payload + descriptors, write table
    del arena, pairs, out
    torch.cuda.empty_cache()
    return {"value": round(world * total / (wall / steps) / GIB, 3), "unit": "GiB/s",
            "ms_per_step": round(wall / steps * 1e3, 4), "records": n, "out_bytes": total,
            "roofline_frac": round(alg / (mean_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "achieved_GBs": round(alg / (mean_ms * 1e-3) / 1e9, 2), "parity_ok": bool(ok)}


def host_leg(torch, eng, sst, n, world, reps=3):
    """Host-inclusive rates (north_star: the path starts and ends in host
    memory): hg_decode_host of the cfg2 table (1 GiB in, 130 MB of spans
    out) and hg_encode_host of the cfg3 arena (2.88 GB + 240 MB of pairs
    in, 3.04 GB out), each from pageable buffers (threaded copies through
    pinned staging) and from page-locked ones (direct DMA).  Median of
    `reps` calls, wall clock around the synchronous ABI call."""
    import ctypes
    from horreum_amd import synth
    from horreum_amd.abi import HgErr
    lib, ctx = eng.lib, eng.ctx

    def vp(a):
        return ctypes.c_void_p(a.ctypes.data)

    def med(fn):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[len(ts) // 2]

    out = {"threads": int(os.environ.get("HG_HOST_COPY_THREADS", "8")), "reps": reps}
    L = sst.numel()
    for mode in ("pageable", "pinned"):
        if mode == "pinned":
            h_t = torch.empty(L, dtype=torch.uint8).pin_memory()
            h_t.copy_(sst)
            sp_t = torch.empty(n * 16, dtype=torch.uint8).pin_memory()
            h, sp = h_t.numpy(), sp_t.numpy()
        else:
            h = sst.cpu().numpy().copy()
            sp = np.empty(n * 16, dtype=np.uint8)
        nn, err = ctypes.c_uint64(), HgErr()

        def dec():
            rc = lib.hg_decode_host(ctx, vp(h), L, vp(sp), n, ctypes.byref(nn), ctypes.byref(err))
            assert rc == 0 and nn.value == n, (rc, nn.value)

        t = med(dec)
        ok = bool(np.array_equal(sp.view("<u8")[0:2 * n:2][:1000],
                                 np.arange(1000, dtype=np.uint64) * 132))
        out[f"decode_cfg2_{mode}"] = {"GiB_s": round(L / t / GIB, 3), "ms": round(t * 1e3, 2),
                                      "parity_spot": ok}
        del h, sp
        if mode == "pinned":
            del h_t, sp_t
    torch.cuda.empty_cache()
    # encode: cfg3 arena -> SSTable bytes
    nE, k, v = 10_000_000, 32, 256
    arena_d, pairs_d = synth.fixed_arena(nE, k, v, seed=3, device=sst.device)
    total = nE * (16 + k + v)
    for mode in ("pageable", "pinned"):
        if mode == "pinned":
            a_t = torch.empty(arena_d.numel(), dtype=torch.uint8).pin_memory()
            a_t.copy_(arena_d)
            p_t = torch.empty(pairs_d.numel(), dtype=torch.uint8).pin_memory()
            p_t.copy_(pairs_d)
            o_t = torch.empty(total, dtype=torch.uint8).pin_memory()
            ha, hp, ho = a_t.numpy(), p_t.numpy(), o_t.numpy()
        else:
            ha, hp = arena_d.cpu().numpy().copy(), pairs_d.cpu().numpy().copy()
            ho = np.empty(total, dtype=np.uint8)
        ol = ctypes.c_uint64()

        def enc():
            rc = lib.hg_encode_host(ctx, vp(ha), ha.size, vp(hp), nE, vp(ho), total,
                                    ctypes.c_void_p(0), 0, ctypes.c_void_p(0), ctypes.byref(ol))
            assert rc == 0 and ol.value == total, (rc, ol.value)

        t = med(enc)
        ok = bool(np.array_equal(ho[16:16 + k + v], ha[:k + v]))
        out[f"encode_cfg3_{mode}"] = {"GiB_s": round(total / t / GIB, 3), "ms": round(t * 1e3, 2),
                                      "parity_spot": ok}
        del ha, hp, ho
        if mode == "pinned":
            del a_t, p_t, o_t
    del arena_d, pairs_d
    torch.cuda.empty_cache()
    # raw pinned DMA rates for reference
    hb = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    db = torch.empty(1 << 30, dtype=torch.uint8, device=sst.device)
    torch.cuda.synchronize()
    t = med(lambda: (db.copy_(hb, non_blocking=True), torch.cuda.synchronize()))
    out["h2d_pinned_GiB_s"] = round(1 / t, 2)
    t = med(lambda: (hb.copy_(db, non_blocking=True), torch.cuda.synchronize()))
    out["d2h_pinned_GiB_s"] = round(1 / t, 2)
    del hb, db
    torch.cuda.empty_cache()
    return out


def cold_open_leg(eng, bufs, lens, caps, reps=3, block_stride=64):
    """Opening a directory of this GPU's 32 cfg 4 tables from files
    (src/sstable/manager.rs:47-55): SSTableManager lists the directory, mmaps
    every file, decodes all of them by one batched launch chain
    (hg_multi_decode_host: H2D through pinned staging, decode, spans D2H) and
    builds each table's block index from its spans.  Wall clock of the constructor, median of `reps`; the files were
    just written, so the page cache is warm (dropping it needs root)."""
    import shutil
    import tempfile
    from horreum_amd.manager import SSTableManager
    d = tempfile.mkdtemp(prefix="hg_cold_open_")
    try:
        for i, b in enumerate(bufs):
            b.cpu().numpy().tofile(os.path.join(d, f"table_{i:03d}"))
        total = sum(lens)
        ts, ok = [], True
        for _ in range(reps):
            t0 = time.perf_counter()
            m = SSTableManager(d, block_stride, 100, engine=eng)
            ts.append(time.perf_counter() - t0)
            ok = ok and len(m.tables) == len(bufs) and all(
                t.get_size() == ln - 16 * n for t, ln, n in zip(m.tables, lens, caps))
            for t in m.tables:
                t.file.unmap()
            del m
        t = sorted(ts)[len(ts) // 2]
        # the same files page-locked first (PersistedFile.pin): registration time
        from horreum_amd.table import PersistedFile
        files = [PersistedFile.open(os.path.join(d, f)) for f in sorted(os.listdir(d))]
        t0 = time.perf_counter()
        for f in files:
            f.pin(eng)
        t_pin = time.perf_counter() - t0
        for f in files:
            f.unmap()
        return {"tables": len(bufs), "bytes": total, "ms": round(t * 1e3, 2),
                "GiB_s": round(total / t / GIB, 3), "page_cache": "warm",
                "steps": "listdir, mmap per file, one batched decode (H2D through pinned "
                         "staging + decode + spans D2H), block index per table",
                "pin_all_ms": round(t_pin * 1e3, 2),
                "pin_note": "hg_host_register of the same 32 mappings (not part of the open: "
                            "pinning costs more than it saves for a file moved once)",
                "parity_spot": bool(ok)}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def multi_table_leg(torch, eng, device, args, world, rank, tables_per_gpu=32, host=False):
    """BASELINE config 4, this GPU's shard: 256 tables of <= 64 MiB (16 B
    sorted keys, values uniform in [8, 4096] B, ~5 % tombstones, seed
    4 + table) round-robin over 8 GPUs -> 32 tables per GPU, decoded by one
    batched call (hg_decode_batch_dev_async: tables fan out over auxiliary
    streams; device resident)."""
    from horreum_amd import synth
    tabs, layouts = [], []
    for i in range(tables_per_gpu):
        t = rank + world * i if world > 1 else i
        v = synth.mixed_table_vlens(64 << 20, 8, 4096, 0.05, seed=4 + t)
        keys = np.arange(v.size, dtype=np.uint64) * 7 + t
        buf, offs = synth.keyed_table(keys, v, seed=4 + t, device=device)
        tabs.append((buf, v.size))
        layouts.append(synth.span_rows(offs[:-1], np.full(v.size, 16), v))
    total = sum(b.numel() for b, _ in tabs)
    spans = [eng.empty(n * 16) for _, n in tabs]
    res = eng.empty(24 * len(tabs))
    bufs = [b for b, _ in tabs]
    lens = [b.numel() for b in bufs]
    caps = [n for _, n in tabs]

    def step():
        eng.decode_batch_dev_async(bufs, lens, spans, caps, res)

    steps = max(1, args.steps // 4)
    wall, ms = time_async(torch, step, steps, 1, world, device)
    r = res.cpu().numpy()
    ok = all(int(r[24 * i:24 * i + 8].view("<u8")[0]) == n and
             int(r[24 * i + 8:24 * i + 12].view("<i4")[0]) == 0 for i, (_, n) in enumerate(tabs))
    for i, want in enumerate(layouts):  # every span of every table, by generator truth
        got = spans[i][: want.shape[0] * 16].cpu().numpy().view("<u8").reshape(-1, 2)
        ok = ok and bool(np.array_equal(got, want))
    recs = sum(n for _, n in tabs)
    mean_ms = sum(ms) / len(ms)
    cold = None
    if host:
        try:
            cold = cold_open_leg(eng, bufs, lens, caps)
        except Exception as e:  # noqa: BLE001 -- a host-path failure must not lose the bench line
            cold = {"error": repr(e)}
    del tabs, spans, bufs, layouts
    torch.cuda.empty_cache()
    return {"value": round(aggregate(wall, steps, world, total), 3), "unit": "GiB/s",
            "cold_open": cold,
            "tables_per_gpu": tables_per_gpu, "bytes_per_gpu": total, "records_per_gpu": recs,
            "ms_per_step": round(wall / steps * 1e3, 4),
            "alg_GBs": round((total + 16 * recs) / (mean_ms * 1e-3) / 1e9, 1),
            "alg_GBs_note": "table bytes + spans per second; hop mode reads ~1 cache line "
                            "per ~2 KiB record, so this is not an HBM fraction",
            "parity_ok": bool(ok), "parity": "counts, kinds and every span of all tables vs "
                                              "the generated record layout"}


def multi_split_leg(torch, eng, devices, ntab=8, per_table=1_000_000, decode_tables=16):
    """SURVEY §8e's split across GPUs, run from ONE process over contexts on
    `devices` (rank 0, while the other ranks wait at a barrier): the cfg 5
    scaled compaction (8 tables x per_table records over the whole key space,
    table t resident on devices[t % G]) by hg_multi_compact_dev -- splitter
    keys sampled from every table, each table decoded in place on its owner,
    every key range's slices gathered to its context by peer copies over
    xGMI (device copies when two contexts share a GPU), merged and encoded
    there -- against one context's hg_compact_dev of the same tables: the
    slices concatenated must equal it byte for byte.  Then cfg 4-shaped
    tables (64 MiB each, 8 B-4 KiB values) from host memory round-robin over
    the contexts by hg_multi_decode_host (PCIe-inclusive), spans checked by
    generator truth.  Wall clock, median of 3."""
    from horreum_amd import synth
    from horreum_amd.multi import MultiEngine
    G = len(devices)
    dev0 = torch.device("cuda", devices[0])
    keys = cfg5_rank_keys(0, ntab, per_table)
    tabs0, owner = [], []
    for t, k in enumerate(keys):
        buf, _ = synth.keyed_table(k, np.full(k.size, 100), seed=cfg5_value_seed(0, t), device=dev0)
        tabs0.append(buf)
        owner.append(t % G)
    sizes = [b.numel() for b in tabs0]
    total = sum(sizes)
    # reference: one context (device 0), the tables in one arena
    offs, acc = [], 0
    for sz in sizes:
        offs.append(acc)
        acc += (sz + 7) & ~7
    arena = torch.zeros(acc, dtype=torch.uint8, device=dev0)
    for o, b in zip(offs, tabs0):
        arena[o:o + b.numel()] = b
    ref = eng.empty(acc)
    c = eng.compact_dev(arena, offs, sizes, ref)
    assert c.status == 0, c
    ref_len = c.data.numel()

    def sync_all():
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)

    def med3(fn):
        fn()
        sync_all()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = fn()
            sync_all()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[1], r

    t_single, _ = med3(lambda: eng.compact_dev(arena, offs, sizes, ref))
    del arena
    tabs = [b.to(torch.device("cuda", devices[o])) for b, o in zip(tabs0, owner)]
    del tabs0
    outs = [torch.zeros(total, dtype=torch.uint8, device=torch.device("cuda", d)) for d in devices]
    m = MultiEngine(devices)
    try:
        t_multi, (rc, ol, orc, res) = med3(lambda: m.compact_dev(tabs, owner, outs))
        phases = m.last_phases()  # of the last of the timed calls
        got_len = sum(int(x) for x in ol)
        ok = rc == 0 and got_len == ref_len
        pos = 0
        for g in range(G):
            if not ok:
                break
            n = int(ol[g])
            ok = torch.equal(outs[g][:n].to(dev0), ref[pos:pos + n])
            pos += n
        slices = [int(x) for x in ol]
        del tabs, outs
        torch.cuda.empty_cache()
        # many tables from host memory, round-robin over the contexts
        host, layouts = [], []
        for t in range(decode_tables):
            v = synth.mixed_table_vlens(64 << 20, 8, 4096, 0.05, seed=4 + t)
            kk = np.arange(v.size, dtype=np.uint64) * 7 + t
            buf, offs_t = synth.keyed_table(kk, v, seed=4 + t, device=dev0)
            host.append(buf.cpu().numpy())
            layouts.append(synth.span_rows(offs_t[:-1], np.full(v.size, 16), v))
            del buf
        hbytes = sum(h.size for h in host)
        t_dec, douts = med3(lambda: m.decode_tables(host))
        dec_ok = all(o.kind == 0 and o.n == w.shape[0] and
                     np.array_equal(o.spans.view("<u8").reshape(-1, 2), w)
                     for o, w in zip(douts, layouts))
    finally:
        m.close()
    return {"contexts": G, "devices": list(devices),
            "distinct_gpus": len(set(devices)),
            "compact": {"api": "hg_multi_compact_dev", "tables": ntab,
                        "records_per_table": per_table, "input_bytes": total,
                        "ms": round(t_multi * 1e3, 3),
                        "GiB_s": round(total / t_multi / GIB, 3),
                        "single_context_ms": round(t_single * 1e3, 3),
                        "slice_bytes": slices, "parity_bytes_ok": bool(ok),
                        "per_context_ms": phases,
                        "waiting_ranks": "gloo side group (CPU): no RCCL kernel on the GPUs",
                        "parity": "slices concatenated == one context's hg_compact_dev"},
            "decode_host": {"api": "hg_multi_decode_host", "tables": decode_tables,
                            "bytes": hbytes, "ms": round(t_dec * 1e3, 3),
                            "GiB_s": round(hbytes / t_dec / GIB, 3),
                            "parity_ok": bool(dec_ok),
                            "note": "pageable host tables: H2D-bound on each GPU's PCIe link"}}


def cfg5_rank_keys(rank, ntab, per_table):
    """Key ids (sorted, unique uint64; 16-byte big-endian keys) of key range
    [rank * 2^40, (rank + 1) * 2^40) of each of the ntab cfg 5 tables: a
    quarter of the keys shared by every table, the rest the table's own."""
    rng = np.random.default_rng(5 + 1000 * rank)
    lo = np.uint64(rank) << np.uint64(40)
    shared = np.unique(rng.integers(0, 1 << 40, size=per_table // 4, dtype=np.uint64)) + lo
    out = []
    for _ in range(ntab):
        own = rng.integers(0, 1 << 40, size=per_table - shared.size, dtype=np.uint64) + lo
        out.append(np.unique(np.concatenate([shared, own])))
    return out


def cfg5_value_seed(rank, t):
    """Seed of the value bytes of table t's slice on `rank`."""
    return 50 + t + 1000 * rank


def compaction_leg(torch, eng, device, world, rank, ntab=8, per_table=1_000_000, host=False,
                   pmc_name=f"{PMC_TAG}_pmc_compaction.json", exact=False, pinned=False):
    """BASELINE config 5 on this GPU's key range: 8 sorted tables of
    `per_table` records each (16 B keys / 100 B values, 132 B records), 25 %
    of each table's keys shared by all tables.  The global dataset is 8
    tables over the key space [0, world * 2^40); rank r holds key range
    [r * 2^40, (r + 1) * 2^40) of every table -- the split by key range of
    SURVEY §8e, its splitters the range boundaries (the first keys of the
    blocks at the cuts) -- so each GPU compacts its slices with no data
    movement and the compacted table is the ranks' outputs in rank order.
    per_table = 8,134,407 (1 GiB of records per table) is one GPU's share of
    cfg 5's 8 x 8 GiB over 8 GPUs.  Decode all, device merge (newest wins),
    encode: one hg_compact_dev call, timed end to end (its host sync for the
    record counts -- the merge is launched from them -- and the final one
    included), median of 3.  Parity: the record count equals the distinct
    keys; with `exact`, the output equals, byte for byte, the rows of the
    key union each taken from the newest table holding it (a stable sort of
    (key, table), gathered on the device).  With `host`, also the end-to-end
    rate from host memory (hg_compact_host on pageable copies: H2D of every
    table, decode, merge, encode, D2H of the compacted table), median of 3."""
    from horreum_amd import synth
    bufs, offs_b, total, n_in, allkeys = [], [], 0, 0, []
    for t, keys in enumerate(cfg5_rank_keys(rank, ntab, per_table)):
        n_in += int(keys.size)
        allkeys.append(keys)
        buf, _ = synth.keyed_table(keys, np.full(keys.size, 100), seed=cfg5_value_seed(rank, t),
                                   device=device)
        bufs.append(buf)
    sizes = [b.numel() for b in bufs]
    hosts = [b.cpu().numpy() for b in bufs] if host else None
    for sz in sizes:
        offs_b.append(total)
        total += (sz + 7) & ~7
    arena = torch.zeros(total, dtype=torch.uint8, device=device)
    for o, b in zip(offs_b, bufs):
        arena[o:o + b.numel()] = b
    want_rows = None
    if exact:  # newest-wins union: stable sort of (key, table)
        allk = np.concatenate(allkeys)
        row = np.concatenate([np.arange(k.size, dtype=np.int64) + base for k, base in
                              zip(allkeys, np.cumsum([0] + [k.size for k in allkeys[:-1]]))])
        order = np.argsort(allk, kind="stable")
        ks = allk[order]
        first = np.ones(ks.size, bool)
        first[1:] = ks[1:] != ks[:-1]
        want_rows = torch.from_numpy(row[order][first]).to(device)
        del allk, row, order, ks, first
    else:
        del bufs
    out = eng.empty(total)

    paths = []  # the merge path of every call (hg_merge_result table / index)

    def run():
        c = eng.compact_dev(arena, offs_b, sizes, out)
        assert c.status == 0, c
        paths.append([int(c.table), int(c.index)])
        return c, c.data.numel()

    run()
    torch.cuda.synchronize(device)
    times = []
    for _ in range(3):
        barrier(world, device)
        t0 = time.perf_counter()
        m, out_len = run()
        torch.cuda.synchronize(device)
        times.append(time.perf_counter() - t0)
    wall = max_over_ranks(sorted(times)[1], world, device)
    in_bytes = sum(sizes)
    n_distinct = int(np.unique(np.concatenate(allkeys)).size)
    exact_ok = None
    del arena  # the check needs the tables' rows and the output only
    torch.cuda.empty_cache()
    if want_rows is not None:
        rows = torch.cat(bufs).view(-1, 132)
        del bufs
        exact_ok = out_len == want_rows.numel() * 132
        step = 1 << 24  # rows per compared slice (no whole-output temporary)
        for i in range(0, want_rows.numel(), step):
            if not exact_ok:
                break
            j = min(i + step, want_rows.numel())
            exact_ok = torch.equal(out[i * 132:j * 132], rows.index_select(0, want_rows[i:j]).view(-1))
        exact_ok = bool(exact_ok)
        del rows, want_rows
    want_first = want_last = None
    if hosts is not None:  # the host leg's parity spot: both ends of the device output
        mib = min(1 << 20, int(out_len))
        want_first = out[:mib].cpu().numpy()
        want_last = out[int(out_len) - mib:int(out_len)].cpu().numpy()
    del out
    torch.cuda.empty_cache()
    line = {"value": round(world * in_bytes / wall / GIB, 3), "unit": "GiB/s of input tables",
            "tables": ntab, "records_per_table": per_table, "input_bytes_per_gpu": in_bytes,
            "merged_records": int(m.n), "merged_bytes": int(out_len),
            "ms": round(wall * 1e3, 3), "times_ms": [round(t * 1e3, 3) for t in times],
            "status": int(m.status), "api": "hg_compact_dev", "input_records": n_in,
            # per call (warm-up first): [0, 0] the parallel merge; [3, k] redone
            # k times after a look-back wait over its budget; [1|2, ..] the
            # reference loop (unsorted input: never here)
            "merge_paths": paths,
            "split": f"key range {rank} of {world} (no data movement between GPUs)",
            # newest wins over sorted unique tables: one record per distinct key
            "parity_count_ok": int(m.n) == n_distinct, "parity_bytes_ok": exact_ok}
    # algorithmic bytes: read the tables, write the compacted table; spans
    # (16 B per input record) and pairs (24 B per output record) each written
    # and read once.  PMC traffic of the same leg from the committed,
    # source-hashed profile.
    alg = in_bytes + int(out_len) + 2 * 16 * n_in + 2 * 24 * int(m.n)
    line["algorithmic_bytes"] = alg
    line["achieved_GBps_alg"] = round(world * alg / wall / 1e9, 1)
    line["roofline_frac"] = round(alg / wall / 1e9 / HBM_PEAK_GBS, 4)
    kern, src = load_leg_pmc(pmc_name, ("hg_decode.hip", "hg_merge.hip", "hg_encode.hip"))
    traffic = sum(v.get("hbm_read_bytes", 0) + v.get("hbm_write_bytes", 0)
                  for v in kern.values()) or None
    line["traffic"] = traffic
    line["traffic_over_algorithmic"] = round(traffic / alg, 3) if traffic else None
    line["traffic_source"] = src
    if hosts is not None:
        hout = np.empty(in_bytes, dtype=np.uint8)  # caller-owned output, reused
        reg = []
        if pinned:  # page-locked in and out: DMA straight from / to them
            for h in hosts + [hout]:
                eng.host_register(h)
                reg.append(h)
        try:
            hpaths = []
            eng.compact_host(hosts, out=hout)  # warm-up (staging buffers, workspaces)
            ht = []
            for _ in range(3):
                t0 = time.perf_counter()
                c = eng.compact_host(hosts, out=hout)
                ht.append(time.perf_counter() - t0)
                hpaths.append([int(c.table), int(c.index)])
            t = sorted(ht)[1]
            # parity spot: the output's first and last MiB against the device run's
            spot = bool(c.status == 0 and c.n == m.n and c.data.size == out_len)
            if spot and want_first is not None:
                spot = (np.array_equal(hout[:want_first.size], want_first)
                        and np.array_equal(hout[out_len - want_last.size:out_len], want_last))
        finally:
            for h in reg:
                eng.host_unregister(h)
        line["host_inclusive"] = {"ms": round(t * 1e3, 2), "GiB_s": round(in_bytes / t / GIB, 3),
                                  "times_ms": [round(x * 1e3, 2) for x in ht],
                                  "input": "pinned (hipHostRegister)" if pinned else "pageable",
                                  "api": "hg_compact_host: H2D of every table, decode, merge, "
                                         "encode, D2H of the compacted table",
                                  "merge_paths": hpaths, "parity_spot": spot}
        del hosts
    return line


if __name__ == "__main__":
    sys.exit(main())
