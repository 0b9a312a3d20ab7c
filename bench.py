"""Headline benchmark: images/sec/node per FL round (+ wall-clock per round), U-Net 256^2, one FL client per GPU.

BASELINE.json metric: "images/sec/node per FL round + wall-clock/round, U-Net 256^2 at 8 clients".
One benchmark *step* is one FL round, exactly as a client runs it (client_fit_model.py:152-174 + fl_server.py:92-105):
  fresh Adam state -> ``epochs`` x (``local_steps`` full training iterations (fwd + bwd + Adam + BN moving stats,
  batch ``batch`` per client, hipGraph replay of the HIP-kernel engine) + a validation pass over the held-out split
  (inference-mode forward, its own hipGraph)) -> FedAvg: weighted RCCL all-reduce of the whole flat model (all 112
  Keras arrays incl. BN moving statistics) across the N clients -> repack weights.
value = N * epochs * local_steps * batch / round_seconds (whole node, training images per round wall-clock; the
validation images are reported separately; weak scaling: per-client work fixed).
Data: synthetic crack images/masks rendered on the device (per-client shard); weights: Keras-default random init.

Launch: ``python bench.py`` (1 GPU); ``python bench.py --gpus N`` spawns the N ranks itself (parallel/spawn.py: one
child process per GPU with the torch.distributed environment, no GPU call in the parent); under
``torchrun --nproc-per-node N bench.py --gpus N`` (WORLD_SIZE set) each process is one rank.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# multi-rank GPU work (RCCL, CUDA-tensor sharing between processes): the host driver only supports dmabuf IPC, so
# the legacy IPC mode must be off - HSA reads this once, at its initialisation, so it is set before this process
# makes any GPU call (with legacy IPC RCCL fails with "hipIpcGetMemHandle: invalid argument")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed FL rounds")
    ap.add_argument("--warmup", type=int, default=1, help="untimed FL rounds")
    ap.add_argument("--img", type=int, default=256)
    ap.add_argument("--batch", type=int, default=16,
                    help="per-client batch (reference: 16; 0 = HBM planner, models/memplan.py)")
    ap.add_argument("--hbm-fraction", type=float, default=0.85, help="HBM share the batch planner may fill")
    ap.add_argument("--epochs", type=int, default=10, help="local epochs per FL round (client_fit_model.py:166)")
    ap.add_argument("--local-steps", type=int, default=0,
                    help="iterations per epoch (0: the reference's Sequence length, 6213 // batch = 388 at batch 16)")
    ap.add_argument("--val-steps", type=int, default=-1,
                    help="validation batches per epoch (-1: the whole held-out split, as Keras fit(validation_data))")
    ap.add_argument("--samples", type=int, default=8000, help="synthetic images per client")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0, help="if >0: run this many single steps and exit")
    ap.add_argument("--profile-eval-steps", type=int, default=0,
                    help="if >0: run this many validation (inference) steps at the bench's eval batch and exit")
    ap.add_argument("--dist-backend", default="nccl",
                    help="process-group backend for N>1 (nccl = RCCL over xGMI; gloo: rehearsal of N ranks "
                         "sharing one GPU, which RCCL refuses)")
    ap.add_argument("--fl", action="store_true",
                    help="also run the FL product path (FLServer + one FLClient per rank over real gRPC, HIP engine, "
                         "RCCL data plane for N>1) for warmup+steps rounds and print a SECOND JSON line: wall-clock "
                         "per round from server release to next release, vs the engine-only round above")
    ap.add_argument("--fedavg-1rank", action="store_true",
                    help="N=1 only: run the overlapped FedAvg path anyway over a 1-rank RCCL group (bucketed "
                         "all-reduce + per-bucket repack on the side stream, first step of the next round waiting "
                         "per layer) - for kernel traces of the overlap (tools/overlap_summary.py)")
    ap.add_argument("--verify-fedavg", action="store_true",
                    help="after the timed rounds, check one weighted FedAvg against an all-gathered reference")
    ap.add_argument("--deterministic", action="store_true",
                    help="deterministic reduction mode (int64 fixed-point cross-block sums: bitwise-reproducible "
                         "steps; models/engine.py UNetEngine(deterministic=True), env CFL_DETERMINISTIC=1)")
    ap.add_argument("--fp8", action="store_true",
                    help="block-scaled fp8 (e4m3, e8m0 per 32 channels) MFMA for every decoder 3x3 conv - ConvT "
                         "forward and data gradient (csrc/kernels/fp8.hip; BASELINE config 5); env CFL_CONV_DTYPE=fp8")
    ap.add_argument("--tune", default="",
                    help="launch-shape knobs for A/B sweeps, 'KEY=V,...' (csrc/kernels/launch.h TuneKey names without "
                         "the TUNE_ prefix, e.g. WGRAD3_BLOCKS=256); default: the built-in heuristics")
    ap.add_argument("--spawn-timeout", type=float, default=0.0,
                    help="self-launch only (--gpus N > 1 without WORLD_SIZE): seconds before the ranks are stopped "
                         "(0: no limit)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N ranks here (fresh child processes, one per GPU) and relay rank 0's JSON line.
        # The parent touches no GPU (device_count does not initialise HIP on this image) and never execs.
        if args.dist_backend == "nccl":
            import torch
            ndev = torch.cuda.device_count()
            if args.gpus > ndev:
                raise SystemExit(f"bench.py: --gpus {args.gpus} with the nccl (RCCL) backend needs {args.gpus} "
                                 f"visible GPUs, found {ndev} (use --dist-backend gloo to rehearse N ranks on fewer)")
        from crack_detection_federatedlearning_grpc_amd.parallel.spawn import spawn_local_ranks
        return spawn_local_ranks(os.path.abspath(__file__), sys.argv[1:], args.gpus,
                                 timeout=args.spawn_timeout or None)
    if os.environ.get("CFL_BENCH_TUNE"):                 # knob sweeps by name from the environment (tools/gpu/bench_ab.sh)
        args.tune = ",".join(t for t in (args.tune, os.environ["CFL_BENCH_TUNE"]) if t)

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 ranks with "
                         f"torch.distributed.run --nproc-per-node {args.gpus} (one rank per GPU)")
    ndev = torch.cuda.device_count()
    if world > 1 and args.dist_backend == "nccl" and world > ndev:
        raise SystemExit(f"bench.py: {world} RCCL ranks need {world} visible GPUs, found {ndev} (RCCL refuses two "
                         f"ranks on one GPU; --dist-backend gloo rehearses N ranks on fewer)")
    torch.cuda.set_device(local % ndev)               # local % ndev: a gloo rehearsal may share one GPU
    dev = torch.device("cuda", local % ndev)
    from crack_detection_federatedlearning_grpc_amd.parallel.rccl import group_stream_info, init_rccl_group
    if world == 1 and args.fedavg_1rank:
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            fport = so.getsockname()[1]
        init_rccl_group(dev, init_method=f"tcp://127.0.0.1:{fport}", rank=0, world_size=1)
    if world > 1:
        if args.dist_backend == "nccl":
            # RCCL group owning its collective: high-priority stream, PreMulSum pre-scale, channel cap
            init_rccl_group(dev)
        else:
            dist.init_process_group(args.dist_backend)
        print(f"[bench] rank {rank}/{world} local_rank {local} -> {dev} ({torch.cuda.get_device_name(dev)}, "
              f"{ndev} visible), backend {dist.get_backend()}, master "
              f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}", file=sys.stderr, flush=True)

    from crack_detection_federatedlearning_grpc_amd.data.device import make_synthetic_device
    from crack_detection_federatedlearning_grpc_amd.models.engine import UNetEngine
    from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable
    from crack_detection_federatedlearning_grpc_amd.parallel.rccl import FedAvgAllReduce
    from crack_detection_federatedlearning_grpc_amd.train.local import epoch_batches
    from crack_detection_federatedlearning_grpc_amd.utils.trace import phase

    if args.tune:
        from crack_detection_federatedlearning_grpc_amd._native_loader import hip
        C = hip()
        for kv in args.tune.split(","):
            k, v = kv.split("=")
            C.set_tune(getattr(C, "TUNE_" + k.strip().upper()), int(v))
    table = ParamTable()
    plan = None
    if args.batch <= 0:
        from crack_detection_federatedlearning_grpc_amd.models.memplan import plan_batch
        plan = plan_batch(args.img, None, args.hbm_fraction, args.samples)
        args.batch = plan.batch
    if args.local_steps <= 0:                              # reference epoch = 6213 // batch iterations
        args.local_steps = max(1, min(6213, args.samples) // args.batch)
    # reference split: the first 6213 of the ~8k images train, the rest validate (kept in proportion for small sets)
    if rank == 0:
        print(f"[bench] rendering {args.samples} synthetic {args.img}^2 images on the device", file=sys.stderr,
              flush=True)
    data = make_synthetic_device(args.samples, args.img, seed=1000 + rank,
                                 split=min(6213, max(args.batch, int(args.samples * 0.7766))))
    det = args.deterministic or os.environ.get("CFL_DETERMINISTIC", "0") == "1"
    conv_dtype = "fp8" if args.fp8 or os.environ.get("CFL_CONV_DTYPE") == "fp8" else "bf16"
    eng = UNetEngine(table, args.batch, args.img, dev, deterministic=det, conv_dtype=conv_dtype)
    eng.bind_data(data.images, data.masks)
    eng.set_flat(table.init_flat(0))                     # same global init on every client
    agg = None
    if world > 1 or args.fedavg_1rank:
        # first bucket = the encoder's parameters: the next round's first step replays its encoder graph after that
        # bucket alone, the rest of the step after every bucket (UNetEngine.train_step)
        agg = FedAvgAllReduce(eng.flat, table, world, first_bucket=eng.split_at)
        agg.timing = True
    n_local = len(data.train_idx)
    batches = torch.as_tensor(epoch_batches(data.train_idx, args.batch, args.local_steps, seed=rank),
                              dtype=torch.int32, device=dev)
    use_graph = not args.no_graph
    eng.bind_batches(batches)          # each step selects its batch on the device (no per-step host index copy)

    if args.profile_steps:
        eng.set_batch_cursor(0)
        for s in range(args.profile_steps):
            eng.train_step(use_graph)
        torch.cuda.synchronize()
        print(json.dumps({"profile_steps": args.profile_steps, "metrics": eng.read_metrics("train")}))
        return 0

    val_steps = len(data.val_idx) // args.batch if args.val_steps < 0 else args.val_steps
    # the reference's 16-image validation batches, evaluated 3-8 at a time by an inference engine sharing the
    # weights (per-pixel means are batching-invariant: models/engine.py UNetEngine.evaluator)
    vimg = epoch_batches(data.val_idx, args.batch, 0, 0)[:val_steps].reshape(-1) if val_steps else None
    # CFL_OVERLAP_VAL=1: each epoch's validation pass runs on its own stream (parameter snapshot) while the next
    # epoch trains (UNetEngine.overlapped_validation)
    overlap_val = os.environ.get("CFL_OVERLAP_VAL", "0") == "1" and use_graph
    ev = eng.evaluator(eng.eval_batch_for(len(vimg)), snapshot=overlap_val) if val_steps else None
    ev_stream = torch.cuda.Stream(device=dev, priority=int(os.environ.get("CFL_VAL_PRIORITY", "0"))) \
        if overlap_val else None
    vbatches = torch.as_tensor(vimg.reshape(-1, ev.B), dtype=torch.int32, device=dev) if val_steps else None

    if args.profile_eval_steps and val_steps:
        for s in range(args.profile_eval_steps):
            ev.idx.copy_(vbatches[s % vbatches.shape[0]])
            ev.eval_step(use_graph)
        torch.cuda.synchronize()
        print(json.dumps({"profile_eval_steps": args.profile_eval_steps, "eval_batch": ev.B,
                          "metrics": ev.read_metrics("eval")}))
        return 0

    def fl_round() -> None:
        eng.reset_optimizer()                              # fresh Adam per round (client_fit_model.py:155-157)
        for _ep in range(args.epochs):                     # model.fit(epochs=10, validation_data=val_gen)
            with phase("bench/train_epoch"):               # roctx ranges with CFL_ROCTX=1 (utils/trace.py)
                eng.set_batch_cursor(0)                    # this epoch's batches: rows 0.. of the bound table
                for s in range(args.local_steps):
                    eng.train_step(use_graph)
            with phase("bench/validate"):
                if overlap_val and val_steps:
                    eng.overlapped_validation(ev, vbatches, ev_stream, use_graph)
                else:
                    for v in range(vbatches.shape[0] if val_steps else 0):
                        ev.idx.copy_(vbatches[v])
                        ev.eval_step(use_graph)
        if ev_stream is not None:
            torch.cuda.current_stream(dev).wait_stream(ev_stream)   # the round's last validation pass
        if agg is not None:
            # weighted FedAvg over RCCL/xGMI, bucketed in layer order on a side stream; each bucket's layers are
            # repacked to bf16 there and the next round's first step waits per bucket (engine.defer_until: the
            # encoder graph after bucket 0, the rest of the step after all)
            eng.defer_until(agg.average_async(float(n_local), on_bucket=eng.pack_bucket))
        else:
            eng.pack()

    def note(msg: str) -> None:                           # progress on stderr (the JSON result stays on stdout)
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    note(f"engine ready: batch {args.batch} @ {args.img}^2, {args.epochs} x {args.local_steps} steps per round, "
         f"{val_steps} validation batches per epoch")
    for w in range(args.warmup):
        tw = time.perf_counter()
        fl_round()
        torch.cuda.synchronize()
        note(f"warm-up round {w + 1}/{args.warmup}: {time.perf_counter() - tw:.2f} s")
    eng.read_metrics("train")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    n_ar0 = 0
    if agg is not None:            # FedAvg cost inside the timed region only (hipEvents, read after the run)
        n_ar0 = len(agg.timings)
        eng.stall_log = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        fl_round()
        if args.steps > 1 and args.img >= 512:
            note(f"timed round {i + 1}/{args.steps} issued")  # (no sync: timing unaffected)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    m = eng.read_metrics("train")
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    fedavg_stats = {}
    if agg is not None:
        # all-reduces issued inside the timed region (round r's FedAvg, consumed by round r+1's first step)
        timed = agg.timings[n_ar0:]
        agg.timings = timed
        fedavg_stats = agg.timing_summary()
        # exposed FedAvg time per consumed all-reduce: how long round r+1's first step stalled on the compute stream
        # for round r's buckets - its wait before the encoder graph (bucket 0) plus its wait before the rest of the
        # step (every bucket). The first timed step consumes the warm-up's all-reduce across the host barrier (not
        # counted); the timed region's last all-reduce is waited by the closing synchronize.
        st = eng.stall_log
        per = []
        for j in range(1, len(st) // 2):
            if j - 1 < len(timed):
                # the two stall brackets only (advisor r5: issue -> end of the first wait also counted the compute
                # stream's own work queued between the FedAvg issue and that wait)
                (b0, a0), (b1, a1) = st[2 * j], st[2 * j + 1]
                per.append(b0.elapsed_time(a0) + b1.elapsed_time(a1))
        if per and fedavg_stats:
            exp = float(np.mean(per))
            fedavg_stats["allreduce_exposed_ms"] = exp
            tot = fedavg_stats["allreduce_repack_ms"]
            fedavg_stats["overlap_fraction"] = max(0.0, min(1.0, 1.0 - exp / tot)) if tot > 0 else None
        if world > 1:              # MAX over ranks (the slowest rank's collective bounds the round)
            keys = [k for k in ("allreduce_ms", "allreduce_repack_ms", "allreduce_exposed_ms") if k in fedavg_stats]
            t = torch.tensor([fedavg_stats[k] for k in keys], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            fedavg_stats.update({k: float(v) for k, v in zip(keys, t.tolist())})
        fedavg_stats = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in fedavg_stats.items()}
        eng.stall_log = None
    fedavg_err = None
    if args.verify_fedavg and agg is not None:
        # one weighted FedAvg with unequal n_k against sum_k n_k w_k / sum n from all-gathered copies
        eng._await_all()
        n_k = float(n_local + 97 * rank)
        mine = eng.flat.clone()
        allw = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allw, mine)
        ns = torch.tensor([n_k], dtype=torch.float64, device=dev)
        alln = [torch.empty_like(ns) for _ in range(world)]
        dist.all_gather(alln, ns)
        nn = torch.cat(alln)
        ref = sum(w.double() * float(n) for w, n in zip(allw, nn)) / float(nn.sum())
        agg.average(n_k)
        fedavg_err = float((eng.flat.double() - ref).abs().max())
        spread = torch.tensor([float(eng.flat.double().sum())], dtype=torch.float64, device=dev)
        lo, hi = spread.clone(), spread.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        fedavg_err = max(fedavg_err, float(hi - lo) / max(1.0, abs(float(hi))))
    round_s = dt / args.steps
    imgs_per_round = world * args.epochs * args.local_steps * args.batch
    value = imgs_per_round / round_s
    if rank == 0:
        out = {"metric": "images/sec/node per FL round", "value": round(value, 2), "unit": "images/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(round_s * 1000.0, 3), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None,
               "dtype": "bf16" if conv_dtype == "bf16" else "fp8 (block-scaled e4m3 decoder 3x3 convs) + bf16", "data": "synthetic (device-rendered crack masks, random init)",
               "wall_clock_per_round_s": round(round_s, 4),
               "ms_per_iteration": round(round_s * 1000.0 / (args.epochs * args.local_steps), 4),
               "val_images_per_round": world * args.epochs * val_steps * args.batch,
               "eval_batch": ev.B if val_steps else None,
               "peak_hbm_gb_per_client": round(torch.cuda.max_memory_allocated(dev) / 2**30, 3),
               "train_loss": round(m["loss"], 5), "train_accuracy": round(m["accuracy"], 5),
               "dist_backend": (dist.get_backend() if world > 1 else None),
               "deterministic": det, "conv_dtype": conv_dtype,
               **({"rccl": group_stream_info()} if dist.is_initialized() and dist.get_backend() == "nccl" else {}),
               **({"fedavg_max_abs_err": fedavg_err} if fedavg_err is not None else {}),
               **fedavg_stats,
               "config": {"model": "Keras U-Net crack segmentation (client_fit_model.py:92-150, 2,058,145 params)",
                          "img_size": args.img, "global_batch": args.batch * world, "per_client_batch": args.batch,
                          "seq_len": None, "epochs_per_round": args.epochs,
                          "local_steps_per_round": args.epochs * args.local_steps,
                          "parallelism": (f"fedavg-dp{world} (1 FL client per GPU, weighted all-reduce over "
                                          f"{'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()})")
                          if agg is not None else "fedavg-dp1 (no aggregation at N=1: weight repack only)",
                          "graph": use_graph, "memplan": plan.as_dict() if plan else None}}
        print(json.dumps(out), flush=True)
    if args.fl:
        del eng, ev, data
        torch.cuda.empty_cache()
        fl_line = run_fl_bench(args, world, rank, round_s)
        if rank == 0:
            print(json.dumps(fl_line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def run_fl_bench(args, world: int, rank: int, engine_round_s: float) -> dict:
    """The reference's product loop, timed: rank 0 hosts the gRPC FLServer (fl_server.py:107-135,152-207), every
    rank runs one FLClient (fl_client.py:77-175) whose LocalFit trains on the HIP engine with the bench's config
    (client_fit_model.py:152-174); for N>1 the clients' FedAvg is the device-resident RCCL all-reduce (the existing
    process group), rank 0 uploading the average. Per-round wall-clock = the server's RoundRecord span: from the
    release of the previous global (window close for round 1) to this round's aggregation - distribution, local
    fit with validation, upload and FedAvg included."""
    import socket
    import torch
    import torch.distributed as dist
    from crack_detection_federatedlearning_grpc_amd import config as C
    from crack_detection_federatedlearning_grpc_amd.fl.client import FLClient
    from crack_detection_federatedlearning_grpc_amd.fl.server import FLServer
    from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable
    from crack_detection_federatedlearning_grpc_amd.train.factory import make_trainer
    rounds = args.warmup + args.steps
    split = min(6213, max(args.batch, int(args.samples * 0.7766)))
    cfg = C.from_args(None, preset="gpu1-256", img_size=args.img, batch_size=args.batch, epochs=args.epochs,
                      steps_per_epoch=args.local_steps, synthetic_samples=args.samples, val_samples=split,
                      max_rounds=rounds, num_clients=world, register_window_s=120.0, codec="flat",
                      data_plane="rccl" if world > 1 else "grpc", client_weight_file="", server_weight_file="",
                      predict_round=0, use_graph=not args.no_graph,
                      work_dir="/tmp", data_seed=7)
    port = torch.zeros(1, dtype=torch.int64, device="cuda")
    srv = None
    if rank == 0:
        srv = FLServer(cfg, table=ParamTable())
        port.fill_(srv.start(0))
    if world > 1:
        dist.all_reduce(port)                                         # server port -> every rank
    host = os.environ.get("MASTER_ADDR", "127.0.0.1") if world > 1 else "127.0.0.1"
    agg_factory = None
    if world > 1:
        from crack_detection_federatedlearning_grpc_amd.parallel.rccl import RcclAggregator
        agg_factory = lambda info: RcclAggregator.from_ready_info(info, cfg)  # noqa: E731 (reuses the group)
    client = FLClient(cfg, lambda: make_trainer(cfg, f"bench{rank}", rank), name=f"bench{rank}",
                      target=f"{host}:{int(port.item())}", aggregator_factory=agg_factory)
    state = client.run()
    out = {}
    if rank == 0:
        srv.done.wait(30)
        srv.stop()
        recs = srv.state.history[args.warmup:]
        spans = [r.t_end - r.t_start for r in recs]
        fl_round_s = sum(spans) / max(1, len(spans))
        hist = client.history[args.warmup:]
        train_s = sum(h["train_s"] for h in hist) / max(1, len(hist))
        ph = [p for p in client.phases if p["round"] > args.warmup]
        mean = lambda k: round(sum(p[k] for p in ph) / max(1, len(ph)), 4)  # noqa: E731
        imgs = world * args.epochs * args.local_steps * args.batch
        out = {"metric": "FL product path: wall-clock per round (server release -> next release, gRPC)",
               "value": round(fl_round_s, 4), "unit": "s/round", "higher_is_better": False, "n_gpus": world,
               "steps": len(spans), "warmup": args.warmup, "final_state": state,
               "images_per_s": round(imgs / fl_round_s, 2), "engine_round_s": round(engine_round_s, 4),
               "control_plane_overhead_s": round(fl_round_s - engine_round_s, 4),
               "client_train_round_s": round(train_s, 4), "client_aggregate_s": mean("aggregate_s"),
               "client_upload_s": mean("upload_s"), "client_wait_s": mean("wait_s"),
               "payload_bytes": ph[-1]["payload_bytes"] if ph else None, "codec": cfg.codec,
               "data_plane": cfg.data_plane, "round_spans_s": [round(x, 4) for x in spans]}
    return out


if __name__ == "__main__":
    sys.exit(main())
