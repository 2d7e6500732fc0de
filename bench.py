"""bench.py — device-resident deserialize throughput of RedRock value blobs on MI355X.

Headline (BASELINE.json metric): GiB/s (+ values/s) of decoding a 1M-value mixed batch
(config-4 proportions) that is already resident in HBM, per GPU, weak-scaled:
each rank owns its own pre-sharded 1M batch (values are independent, so there is no data-path
collective), and `value` = all ranks' blob bytes / max-over-ranks time.

A step = one rr_decode_batch call (look-back reset + one decode launch) over the whole batch.
Also reported: encode throughput (same batch), the roofline of the decode kernel (algorithmic
bytes per launch / launch time vs 8 TB/s HBM3E) and, on rank 0 at N=1, the CPU baseline: the
reference-faithful desObject restatement (oracle/rro_faithful.c) on the box's host cores.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--n VALUES] [--config 4]
Multi-GPU: `python bench.py --gpus N` starts its N ranks itself (one process per GPU, a
torch.distributed.run child process started before anything touches the GPU; this process only
waits for it and exits with its code), or run it under an outside launcher:
python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
(WORLD_SIZE must then equal --gpus).  `--plan-only` prints the launch decision and the rank
layout without any GPU call; `--launch-check` runs the N ranks over gloo on the CPU and has rank
0 print the ranks that joined (tests/test_bench_launch.py).
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s + values/s device-resident serdes, 1M mixed batch @1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
CONFIG_NAMES = {1: "100K 64-byte RAW strings", 2: "1M Zipf 16B-4KiB strings", 3: "1M hash ziplists x16 pairs",
                4: "1M mixed String/List/Set/Hash/ZSet (config-4 proportions)",
                5: "config 5: shards of a 100M mixed batch (config-4 proportions), byte-balanced 8-way plan"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--n", type=int, default=1_000_000, help="values per GPU")
    p.add_argument("--config", type=int, default=4)
    p.add_argument("--total", type=int, default=100_000_000, help="config 5: values in the whole batch")
    p.add_argument("--shards", type=int, default=8, help="config 5: shards of the byte-balanced plan")
    p.add_argument("--shard-index", type=int, default=None,
                   help="config 5: the shard this rank decodes (default: its rank; the last shard at N=1)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the CPU baseline leg")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-check", action="store_true")
    p.add_argument("--no-host", action="store_true", help="skip the PCIe-inclusive host leg and the copy reference")
    p.add_argument("--no-split", action="store_true", help="skip the RCCL root split/gather leg")
    p.add_argument("--no-snappy", action="store_true", help="skip the snappy block-compression leg (row f3)")
    p.add_argument("--profile-only", action="store_true", help="decode steps only (for rocprofv3)")
    p.add_argument("--profile-encode", action="store_true", help="one decode, then encode steps only (for rocprofv3)")
    p.add_argument("--plan-only", action="store_true", help="print the launch decision and rank layout, no GPU call")
    p.add_argument("--launch-check", action="store_true",
                   help="start the ranks as the bench would, join them over gloo on the CPU, report who joined")
    p.add_argument("--split-timeout", type=float, default=120.0,
                   help="watchdog on the RCCL split/gather leg: past it every rank exits non-zero")
    p.add_argument("--stall-rank", type=int, default=None,
                   help="--launch-check only: this rank never joins (tests the watchdog's non-zero exit)")
    return p.parse_args()


def launch_plan(gpus, env):
    """How this process runs `--gpus N`: "direct" when it is already one rank of a job (WORLD_SIZE
    set by an outside launcher; it must equal N) or N = 1; "spawn" when it must start the N ranks
    itself.  Returns (plan dict, error string or None).  Pure: no GPU call, no torch import."""
    ws = env.get("WORLD_SIZE")
    if gpus < 1:
        return None, f"--gpus {gpus}: need at least one GPU"
    if ws is not None:
        world = int(ws)
        if world != gpus:
            return None, f"WORLD_SIZE={world} but --gpus {gpus}: the launcher and the bench disagree"
        return {"launch": "direct", "world": world, "rank": int(env.get("RANK", "0")),
                "local_rank": int(env.get("LOCAL_RANK", "0"))}, None
    if gpus == 1:
        return {"launch": "direct", "world": 1, "rank": 0, "local_rank": 0}, None
    return {"launch": "spawn", "world": gpus, "ranks": [{"rank": r, "local_rank": r, "device": f"cuda:{r}"}
                                                         for r in range(gpus)]}, None


def spawn_ranks(gpus, argv):
    """Start `gpus` ranks of this script as one torch.distributed.run child process (a child, not
    an exec: nothing here has touched the GPU, and the ranks are fresh processes), on 127.0.0.1
    with a free port; returns the child's exit code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # (dmabuf IPC only on these hosts)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


WATCHDOG_EXIT = 3   # a collective that hangs fails the job: never rc 0


def arm_watchdog(seconds, rank, on_fire=None):
    """A collective that has not returned after `seconds` fails the job: rank 0 runs `on_fire`
    (prints what it has), then every rank leaves with WATCHDOG_EXIT.  os._exit, because the hung
    thread holds the collective; the exit is non-zero so a launcher (and the driver's SCALE run)
    sees the hang instead of a clean rc 0.  Returns the started timer; cancel() it on success."""
    import threading

    def _bail():
        try:
            if rank == 0 and on_fire is not None:
                on_fire()
            print(f"bench.py: rank {rank}: collective watchdog fired after {seconds:.0f} s, exiting "
                  f"{WATCHDOG_EXIT}", file=sys.stderr, flush=True)
        finally:
            os._exit(WATCHDOG_EXIT)

    dog = threading.Timer(seconds, _bail)
    dog.daemon = True
    dog.start()
    return dog


def launch_check(world, rank, stall_rank=None, timeout=120.0):
    """--launch-check inside a rank: join the job over gloo (no GPU) and report the ranks.  With
    `stall_rank` that rank never enters the all-gather, so the others hang in it: the same watchdog
    as the bench's split/gather leg must end every rank with a non-zero code."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([rank], dtype=torch.int64)
    got = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dog = arm_watchdog(timeout, rank, lambda: print(json.dumps({"launch_check": True, "world": world,
                                                                "error": f"timeout after {timeout:.0f} s"}),
                                                    flush=True))
    if rank == stall_rank:
        time.sleep(10 * timeout + 60)   # the watchdog ends this rank too
    dist.all_gather(got, t)
    dog.cancel()
    if rank == 0:
        print(json.dumps({"launch_check": True, "world": dist.get_world_size(), "n_gpus": world,
                          "ranks": [int(x.item()) for x in got]}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    plan, err = launch_plan(args.gpus, os.environ)
    if err:
        print(f"bench.py: {err}", file=sys.stderr)
        sys.exit(2)
    if args.plan_only:
        print(json.dumps(plan), flush=True)
        return
    if plan["launch"] == "spawn":   # before any GPU call: the ranks are fresh processes
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if args.launch_check:
        launch_check(plan["world"], plan["rank"], args.stall_rank, args.split_timeout)
        return
    import torch
    import torch.distributed as dist

    import redrock_old_amd as rr

    world, rank, local = plan["world"], plan["rank"], plan["local_rank"]
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    # ---- this rank's shard (pre-sharded: distinct seed per rank) ----
    t0 = time.perf_counter()
    shard_info = None
    if args.config == 5:
        # BASELINE config 5: one shard of the byte-balanced plan of the whole 100M batch, generated
        # on its own (seekable generator: sizes of all values, then the shard's bytes)
        nt = min(16, len(os.sched_getaffinity(0)))
        k = args.shard_index if args.shard_index is not None else (rank if world > 1 else args.shards - 1)
        nb_all, nd_all = rr.gen_sizes(5, 0, args.total, nthreads=nt)
        offs_all = np.zeros(args.total + 1, np.uint64)
        np.cumsum(nb_all, out=offs_all[1:])
        del nb_all
        v0, v1, b0, b1 = (int(x) for x in rr.shard_plan(offs_all, args.shards)[k])
        shard_info = {"total_values": args.total, "shards": args.shards, "shard": k, "values": [v0, v1],
                      "bytes": [b0, b1], "whole_batch_bytes": int(offs_all[-1]),
                      "descriptors_before": int(nd_all[:v0].sum(dtype=np.uint64)),
                      "descriptors": int(nd_all[v0:v1].sum(dtype=np.uint64))}
        del offs_all, nd_all
        data, offs = rr.gen_range(5, v0, v1, nthreads=nt)
    else:
        seed = int(rr.lib().rr_gen_default_seed(args.config)) + 7919 * rank
        data, offs = rr.gen_batch(args.config, args.n, seed)
    t_gen = time.perf_counter() - t0
    n = len(offs) - 1
    nb = int(offs[-1])
    types, counts = np.unique(data[offs[:-1].astype(np.int64)], return_counts=True)

    eng = rr.Engine(local)
    eng.reserve(n, nb)
    d_data = torch.from_numpy(data).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    cap = rr.elem_bound(n, nb) if shard_info is None else shard_info["descriptors"]   # (config 5: the exact count)
    d_vals = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    d_elems = torch.empty(cap * 16, dtype=torch.uint8, device=dev)
    d_arena = torch.empty((nb + 15) & ~15, dtype=torch.uint8, device=dev)
    d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
    d_out = torch.empty((nb + 15) & ~15, dtype=torch.uint8, device=dev)
    d_ooffs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_tot2 = torch.zeros(4, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()

    def decode():
        eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot, stream=stream)

    def encode():
        eng.encode_device(d_vals, d_elems, d_arena, d_out, d_ooffs, d_tot2, stream=stream)

    def barrier():
        if world > 1:
            dist.barrier()

    def timed(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        barrier()
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t_start = time.perf_counter()
        ev0.record(stream)
        for _ in range(steps):
            fn()
        ev1.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t_start
        barrier()
        ev_ms = ev0.elapsed_time(ev1) / steps
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()), ev_ms

    if args.profile_only:
        timed(decode, args.steps, args.warmup)
        return
    if args.profile_encode:
        decode()
        timed(encode, args.steps, args.warmup)
        return

    wall_dec, ev_dec = timed(decode, args.steps, args.warmup)
    tot = d_tot.cpu().numpy().view(np.uint64).copy()
    n_elems, n_bad, payload = int(tot[0]), int(tot[2]), int(tot[3])
    wall_enc, ev_enc = timed(encode, args.steps, args.warmup)
    tot2 = d_tot2.cpu().numpy().view(np.uint64).copy()

    # ---- reference legs (not the headline): device copy bandwidth, PCIe-inclusive decode ----
    # the engine's own streaming copy (rr_copy_device: the decode window copy's load/store
    # shape) is the measured ceiling the roofline is also priced against; torch's copy beside it
    d_copy = torch.zeros_like(d_data)
    _, ev_rrcopy = timed(lambda: eng.copy_device(d_copy, d_data, stream=stream), args.steps, args.warmup)
    copy_ok = bool(torch.equal(d_copy, d_data))
    _, ev_copy = timed(lambda: d_copy.copy_(d_data), args.steps, args.warmup)
    del d_copy
    rrcopy_gbs = 2 * d_data.numel() / (ev_rrcopy * 1e-3) / 1e9   # read + write
    copy_gbs = 2 * d_data.numel() / (ev_copy * 1e-3) / 1e9
    copy_ref = {"GBs": round(rrcopy_gbs, 1), "frac_of_peak": round(rrcopy_gbs / HBM_PEAK_GBS, 4),
                "ms": round(ev_rrcopy, 4), "bit_exact": copy_ok,
                "what": "rr_copy_device (the engine's streaming copy kernel) of the blob buffer, read + write bytes",
                "torch_copy_GBs": round(copy_gbs, 1)}
    host = None
    if not args.no_host:
        # one step = pinned H2D of blobs + offsets, the decode, pinned D2H of records,
        # descriptors and arena (what rr_decode_batch_host does, through pinned buffers)
        h_data = torch.from_numpy(data).pin_memory()
        h_offs = torch.from_numpy(offs.view(np.int64)).pin_memory()
        h_vals = torch.empty(d_vals.numel(), dtype=torch.uint8).pin_memory()
        h_elems = torch.empty(n_elems * 16, dtype=torch.uint8).pin_memory()
        h_arena = torch.empty(nb, dtype=torch.uint8).pin_memory()

        def e2e():
            d_data.copy_(h_data, non_blocking=True)
            d_offs.copy_(h_offs, non_blocking=True)
            decode()
            h_vals.copy_(d_vals, non_blocking=True)
            h_elems.copy_(d_elems[: n_elems * 16], non_blocking=True)
            h_arena.copy_(d_arena[:nb], non_blocking=True)

        wall_ser, _ = timed(e2e, 5, 1)
        # the product's host entry point on the same pinned buffers: rr_decode_batch_host
        # (chunked: uploads, per-chunk decodes and downloads on separate streams overlap)
        import ctypes
        L = rr.lib()
        h_tot = rr.Totals()

        def e2e_api():
            rc = L.rr_decode_batch_host(eng._ctx, h_data.data_ptr(), h_offs.data_ptr(), n, h_vals.data_ptr(),
                                        h_elems.data_ptr(), n_elems, h_arena.data_ptr(), ctypes.byref(h_tot))
            assert rc == 0, "rr_decode_batch_host failed"

        wall_api, _ = timed(e2e_api, 5, 1)

        def e2e_records():   # arena = NULL: the caller's blob buffer is the arena (the mirror)
            rc = L.rr_decode_batch_host(eng._ctx, h_data.data_ptr(), h_offs.data_ptr(), n, h_vals.data_ptr(),
                                        h_elems.data_ptr(), n_elems, None, ctypes.byref(h_tot))
            assert rc == 0, "rr_decode_batch_host failed"

        wall_rec, _ = timed(e2e_records, 5, 1)
        e2e_api()   # (the arena back on the host for the encode leg)
        api_ok = (int(h_tot.n_elems) == n_elems and int(h_tot.payload) == payload
                  and torch.equal(h_vals, d_vals.cpu()) and torch.equal(h_elems, d_elems[: n_elems * 16].cpu()))
        # dump direction from host memory: rr_encode_batch_host on the decoded flat batch
        h_out = torch.empty((nb + 15) & ~15, dtype=torch.uint8).pin_memory()
        h_ooffs = torch.empty(n + 1, dtype=torch.int64).pin_memory()
        h_tot2 = rr.Totals()

        def e2e_encode():
            rc = L.rr_encode_batch_host(eng._ctx, h_vals.data_ptr(), h_elems.data_ptr(), n_elems,
                                        h_arena.data_ptr(), nb, n, h_out.data_ptr(), h_out.numel(),
                                        h_ooffs.data_ptr(), ctypes.byref(h_tot2))
            assert rc == 0, "rr_encode_batch_host failed"

        wall_enc_host, _ = timed(e2e_encode, 5, 1)
        enc_ok = bool(torch.equal(h_out[:nb], h_data[:nb])) and int(h_tot2.bytes) == nb
        host = {"host_e2e": {"gib_s": round(nb * 5 / wall_api / 2 ** 30, 2),
                             "ms_per_step": round(wall_api / 5 * 1e3, 3), "matches_device_decode": bool(api_ok),
                             "what": "rr_decode_batch_host on pinned host buffers: blobs+offsets up, decode, "
                                     "records+descriptors+arena down, chunked so the two PCIe directions overlap"},
                "host_e2e_blob_as_arena": {"gib_s": round(nb * 5 / wall_rec / 2 ** 30, 2),
                                           "ms_per_step": round(wall_rec / 5 * 1e3, 3),
                                           "what": "the same call with arena = NULL: records and descriptors "
                                                   "come down, the caller's blob buffer serves as the arena"},
                "host_e2e_encode": {"gib_s": round(nb * 5 / wall_enc_host / 2 ** 30, 2),
                                    "ms_per_step": round(wall_enc_host / 5 * 1e3, 3), "roundtrip_bit_exact": enc_ok,
                                    "what": "rr_encode_batch_host on pinned host buffers: records+descriptors+arena "
                                            "up, encode, blobs+offsets down, chunked so uploads, encodes and downloads overlap"},
                "host_e2e_serial": {"gib_s": round(nb * 5 / wall_ser / 2 ** 30, 2),
                                    "ms_per_step": round(wall_ser / 5 * 1e3, 3),
                                    "what": "the same transfers in one stream, back to back (no overlap)"}}
        del h_data, h_offs, h_vals, h_elems, h_arena, h_out, h_ooffs

    # ---- correctness of what was timed ----
    parity = None
    if not args.no_check:
        rt = bool(torch.equal(d_out[:nb], d_data[:nb])) and bool(
            np.array_equal(d_ooffs.cpu().numpy().view(np.uint64), offs))
        parity = {"roundtrip_bit_exact": rt, "n_bad": n_bad}
        if rank == 0 and world == 1:
            from oracle import cpu
            ov, oe, _, ot = cpu.decode(data, offs, elem_cap=n_elems, nthreads=min(16, cpu.nprocs()))
            v = d_vals.cpu().numpy().view(rr.VALUE_DT)
            e = d_elems[: n_elems * 16].cpu().numpy().view(rr.ELEM_DT)
            parity["decode_vs_oracle_bit_exact"] = bool(np.array_equal(v, ov) and np.array_equal(e, oe))

    # ---- aggregate over ranks ----
    agg = torch.tensor([nb, n, n_elems, payload], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(agg)
    tot_bytes, tot_vals = float(agg[0]), float(agg[1])
    ms_step = wall_dec / args.steps * 1e3
    gib_s = tot_bytes * args.steps / wall_dec / 2 ** 30
    vals_s = tot_vals * args.steps / wall_dec
    enc_gib_s = tot_bytes * args.steps / wall_enc / 2 ** 30

    # roofline of the decode kernel (SURVEY.md §8d algorithmic bytes, per launch, this rank)
    alg_bytes = nb + 16 * n + 16 * n_elems + payload
    traffic = measured_traffic(args.config, n, nb)
    achieved = alg_bytes / (ev_dec * 1e-3) / 1e9
    enc_alg = 16 * n + 16 * n_elems + int(tot2[3]) + nb + 8 * (n + 1)
    enc_achieved = enc_alg / (ev_enc * 1e-3) / 1e9

    result = {
        "metric": METRIC,
        "value": round(gib_s, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded C generator, SURVEY.md §8d shapes)",
        "config": {"workload": f"device-resident decode, {CONFIG_NAMES.get(args.config, args.config)}",
                   "values_per_gpu": n, "blob_bytes_per_gpu": nb, "descriptors_per_gpu": n_elems,
                   "parallelism": f"shard{world} (pre-sharded, no data-path collective)",
                   "type_histogram": {int(t): int(c) for t, c in zip(types, counts)},
                   **({"config5_shard": shard_info} if shard_info else {})},
        "values_per_s": round(vals_s, 1),
        "decode": {"gib_s": round(gib_s, 2), "values_per_s": round(vals_s, 1), "ms_per_step": round(ms_step, 4),
                   "event_ms_per_launch": round(ev_dec, 4)},
        "encode": {"gib_s": round(enc_gib_s, 2), "ms_per_step": round(wall_enc / args.steps * 1e3, 4),
                   "event_ms_per_launch": round(ev_enc, 4),
                   "roofline_achieved_GBs": round(enc_achieved, 1)},
        "roofline": {"bound": "hbm", "kernel": "rr_decode_batch (count_kernel + decode_kernel)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic[0],
                     "traffic_source": traffic[1],
                     "alg_bytes_per_launch": alg_bytes,
                     "frac_of_copy": round(achieved / copy_ref["GBs"], 4) if copy_ref["GBs"] else None},
        "copy_ref": copy_ref,
        "parity": parity,
        **(host or {}),
        "gen_s": round(t_gen, 2),
    }

    if not args.no_split:
        # a hang in a collective must not hide the headline line, nor pass as success: after
        # --split-timeout rank 0 prints what it has and every rank exits WATCHDOG_EXIT
        def _report():
            result["split_gather"] = {"error": f"timeout after {args.split_timeout:.0f} s"}
            print(json.dumps(result), flush=True)

        dog = arm_watchdog(args.split_timeout, rank, _report)
        try:
            result["split_gather"] = split_gather_leg(rr, torch, dist, eng, world, rank, dev, stream, d_data, d_offs,
                                                      d_vals, d_elems, n, nb, n_elems)
        except Exception as ex:   # reported, never fatal to the headline
            result["split_gather"] = {"error": repr(ex)[:300]}
        dog.cancel()

    if not args.no_snappy:
        try:
            result["snappy"] = snappy_leg(rr, torch, eng, stream, d_data, nb, timed, args,
                                          cpu_too=(rank == 0 and world == 1 and not args.no_cpu))
        except Exception as ex:   # reported, never fatal to the headline
            result["snappy"] = {"error": repr(ex)[:300]}

    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(data, offs, nb, args.cpu_seconds)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def split_gather_leg(rr, torch, dist, eng, world, rank, dev, stream, d_data, d_offs, d_vals, d_elems, n, nb,
                     n_elems):
    """Root split / gather through the C library's RCCL entry points (rr_split_plan, rr_split,
    rr_gather), reported separately from the device-resident headline: rank 0's
    batch is cut into `world` byte-balanced shards and scattered over xGMI, every rank decodes
    its shard, and the decoded shards are gathered back to rank 0, where they must equal rank
    0's whole-batch decode bit for bit."""
    cid = torch.zeros(rr.COMM_ID_BYTES, dtype=torch.uint8, device=dev)
    if rank == 0:
        cid.copy_(torch.frombuffer(bytearray(rr.Comm.new_id()), dtype=torch.uint8))
    if world > 1:
        dist.broadcast(cid, 0)
    comm = rr.Comm(eng, world, rank, bytes(cid.cpu().numpy().tobytes()))
    try:
        def sync():
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()

        def tmax(x):
            t = torch.tensor([x], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())

        root = rank == 0
        plan = comm.split_plan(d_data if root else None, d_offs if root else None, root=0, stream=stream)
        me = plan[rank]
        nv, mb = int(me.v1 - me.v0), int(me.b1 - me.b0)
        m_data = torch.empty(max((mb + 15) & ~15, 16), dtype=torch.uint8, device=dev)
        m_offs = torch.empty(nv + 1, dtype=torch.int64, device=dev)
        cap = rr.elem_bound(nv, mb)
        m_vals = torch.empty(max(nv, 1) * 16, dtype=torch.uint8, device=dev)
        m_elems = torch.empty(max(cap, 1) * 16, dtype=torch.uint8, device=dev)
        m_arena = torch.empty(m_data.numel(), dtype=torch.uint8, device=dev)
        m_tot = torch.zeros(4, dtype=torch.int64, device=dev)
        w_vals = torch.empty(n * 16, dtype=torch.uint8, device=dev) if root else None
        w_elems = torch.empty(max(n_elems, 1) * 16, dtype=torch.uint8, device=dev) if root else None
        t_split, t_dec, t_gather = [], [], []
        for rep in range(4):   # rep 0 warms up
            sync()
            t0 = time.perf_counter()
            plan = comm.split_plan(d_data if root else None, d_offs if root else None, root=0, stream=stream)
            comm.split(plan, d_data if root else None, d_offs if root else None, m_data, m_offs, root=0,
                       stream=stream)
            sync()
            t1 = time.perf_counter()
            eng.decode_device(m_data, m_offs, m_vals[:nv * 16], m_elems, m_arena, m_tot, stream=stream)
            sync()
            t2 = time.perf_counter()
            ne = int(m_tot[0].item())
            comm.gather(plan, m_vals[:nv * 16], m_elems[:ne * 16], ne, w_vals, w_elems, root=0, stream=stream)
            sync()
            t3 = time.perf_counter()
            if rep:
                t_split.append(tmax(t1 - t0))
                t_dec.append(tmax(t2 - t1))
                t_gather.append(tmax(t3 - t2))
        moved = sum(int(p.b1 - p.b0) + 8 * int(p.v1 - p.v0 + 1) for k, p in enumerate(plan) if k != 0)
        out = {"what": f"rank 0's batch split into {world} shards over RCCL (rr_split), decoded per rank, "
                       "gathered to rank 0 (rr_gather); wall ms, max over ranks, median of 3",
               "split_ms": round(statistics.median(t_split) * 1e3, 3),
               "shard_decode_ms": round(statistics.median(t_dec) * 1e3, 3),
               "gather_ms": round(statistics.median(t_gather) * 1e3, 3),
               "split_bytes_sent": moved}
        if root:
            out["gather_bit_exact"] = bool(torch.equal(w_vals, d_vals[:n * 16]) and
                                           torch.equal(w_elems[:n_elems * 16], d_elems[:n_elems * 16]))
        return out
    finally:
        comm.close()


SNAPPY_BLOCK = 16384   # RocksDB data block size the reference configures (rocksdbapi.cc:77,142)


def snappy_leg(rr, torch, eng, stream, d_data, nb, timed, args, cpu_too):
    """Row f3: the same blob bytes cut into 16 KiB RocksDB data blocks, compressed and
    decompressed on the GPU in snappy's raw format (include/rr_snappy.h), device-resident,
    HIP events over the timed steps; round trip checked; the CPU oracle (snappy 1.1.8
    restatement) on a bounded sample beside it."""
    cuts = np.append(np.arange(0, nb, SNAPPY_BLOCK, dtype=np.uint64), np.uint64(nb))
    n = len(cuts) - 1
    d_offs = torch.from_numpy(cuts.view(np.int64)).to(d_data.device)
    cap = int(rr.lib().rr_snappy_compress_bound(n, d_data.numel()))
    d_comp = torch.empty(cap, dtype=torch.uint8, device=d_data.device)
    d_coffs = torch.empty(n + 1, dtype=torch.int64, device=d_data.device)
    d_back = torch.empty(d_data.numel(), dtype=torch.uint8, device=d_data.device)
    d_boffs = torch.empty(n + 1, dtype=torch.int64, device=d_data.device)
    d_st = torch.empty(n, dtype=torch.uint8, device=d_data.device)
    steps, warm = max(1, args.steps // 4), 1
    _, ev_c = timed(lambda: eng.snappy_compress_device(d_data, d_offs, d_comp, d_coffs, stream=stream), steps, warm)
    zb = int(d_coffs[-1].item())
    d_z = d_comp[:((zb + 15) & ~15) or 16]
    _, ev_d = timed(lambda: eng.snappy_decompress_device(d_z, d_coffs, d_back, d_boffs, d_st, stream=stream), steps, warm)
    ok = int(d_st.max().item()) == 0 and bool(torch.equal(d_back[:nb], d_data[:nb]))
    out = {"what": f"{n} blocks of {SNAPPY_BLOCK} B (the decode batch's blobs), snappy raw format, device-resident",
           "compressed_bytes": zb, "ratio": round(zb / nb, 4), "roundtrip_bit_exact": ok,
           "compress": {"ms": round(ev_c, 3), "GBs_input": round(nb / ev_c / 1e6, 1)},
           "decompress": {"ms": round(ev_d, 3), "GBs_output": round(nb / ev_d / 1e6, 1),
                          "hbm_alg_GBs": round((nb + zb) / ev_d / 1e6, 1)}}
    if cpu_too:
        from oracle import cpu
        data = d_data[:nb].cpu().numpy()
        sub = cuts[: min(n, 2048) + 1]
        sb = int(sub[-1])
        for thr in (1, 16):
            _, _, t1 = cpu.snappy_compress_blocks(data, sub, nthreads=thr)
            z, zo, _ = cpu.snappy_compress_blocks(data, sub, nthreads=thr)
            _, _, t2 = cpu.snappy_uncompress_blocks(z, zo, sub, nthreads=thr)
            out[f"cpu_{thr}t"] = {"compress_GBs": round(sb / t1 / 1e9, 2), "decompress_GBs": round(sb / t2 / 1e9, 2)}
        out["cpu_sample"] = f"first {len(sub) - 1} blocks ({sb} B), oracle/rr_snappy.c (snappy 1.1.8 restatement)"
    return out


def measured_traffic(config, n, nb):
    """HBM bytes per decode call from the newest committed rocprofv3 PMC summary of this workload
    (tools/profile_bench.sh + tools/traffic_summary.py) and that file's name — the counters are
    collected in their own runs (rocprofv3 --pmc cannot ride along a timed run), so the line says
    which profile they come from — or (None, None) if none matches."""
    import glob
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_decode_summary.json")), reverse=True):
        try:
            with open(p) as f:
                d = json.load(f)
            w = d.get("workload") or {}
            if (w.get("config"), w.get("n"), w.get("blob_bytes")) == (config, n, nb) and d.get("traffic_bytes_per_call"):
                return int(d["traffic_bytes_per_call"]), os.path.relpath(p, ROOT)
        except (OSError, ValueError):
            continue
    return None, None


def cpu_baseline(data, offs, nb, budget_s):
    """Reference-faithful desObject (one thread, robj/sds/dict/skiplist/quicklist building, as
    rock.c:468 runs it) over the same batch, repeated within ~budget_s; median pass."""
    from oracle import cpu
    n = len(offs) - 1
    # bounded sample: a prefix of the same batch sized to ~1 s per pass
    out = {}
    _, _, _, t_dec, t_enc = cpu.faithful_roundtrip(data[: int(offs[min(n, 20000)]) + 16], offs[: min(n, 20000) + 1])
    per_val = max(t_dec / min(n, 20000), 1e-9)
    m = int(min(n, max(20000, 1.0 / per_val)))
    sub_off = offs[: m + 1]
    sub = data[: ((int(sub_off[-1]) + 15) & ~15)]
    times_d, times_e = [], []
    t_end = time.perf_counter() + budget_s * 0.6
    while len(times_d) < 3 or (time.perf_counter() < t_end and len(times_d) < 9):
        _, _, bad, td, te = cpu.faithful_roundtrip(sub, sub_off)
        times_d.append(td)
        times_e.append(te)
    sb = int(sub_off[-1])
    td = statistics.median(times_d)
    te = statistics.median(times_e)
    out.update({"value": round(sb / td / 2 ** 30, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
                "sample": f"first {m} values ({sb} B) of the same batch, faithful desObject, median of {len(times_d)}",
                "values_per_s": round(m / td, 1), "encode_gib_s": round(sb / te / 2 ** 30, 4)})
    out["per_core_gib_s"] = out["value"]
    # flat restatement (same output as the GPU) on 1 thread, 16 threads (the box's CPU share per
    # GPU) and every core this process may run on (its affinity and cgroup quota; at most 128)
    allc = min(len(os.sched_getaffinity(0)), 128)
    quota = None   # the job's CPU quota (cgroup v2 cpu.max), which bounds any thread count
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    out["cpu_quota_cores"] = quota
    if quota:   # threads past the quota only time-share the same cores
        allc = min(allc, max(1, int(quota)))
    flat = {}
    for thr in sorted({1, min(16, allc), allc}):
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            cpu.decode(sub, sub_off, nthreads=thr)
            ts.append(time.perf_counter() - t0)
        flat[thr] = sb / statistics.median(ts) / 2 ** 30
        out[f"flat_{thr}t_gib_s"] = round(flat[thr], 4)
    out["flat_all_cores"] = {"cores": allc, "gib_s": round(flat[allc], 4),
                             "per_core_gib_s": round(flat[allc] / allc, 4)}
    out["host_cpus"] = cpu.nprocs()
    return out


if __name__ == "__main__":
    main()
