"""All-reduce bandwidth versus bucket size over torch.distributed (RCCL on
MI355X, gloo on CPU) - the bucket-size curve behind
``root.common.engine.dp.bucket_mb`` (docs/PARALLEL.md).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/bench_allreduce.py [--dtype float32] [--iters 20]

Prints one JSON line per size on rank 0: algorithm bandwidth (bytes /
time) and bus bandwidth (x 2 (n-1)/n, the ring-normalised figure RCCL's
own tests report), so xGMI link utilisation can be read directly."""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,4,16,32,64,128,256")
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--backend", default=None)
    args = ap.parse_args()
    gpu = torch.cuda.is_available()
    backend = args.backend or ("nccl" if gpu else "gloo")
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29555")
    if gpu:
        torch.cuda.set_device(local % torch.cuda.device_count())
    dist.init_process_group(backend, rank=rank, world_size=world)
    dev = torch.device("cuda") if gpu else torch.device("cpu")
    dt = getattr(torch, args.dtype)
    esz = torch.tensor([], dtype=dt).element_size()

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    for mb in [float(v) for v in args.sizes_mb.split(",")]:
        n = int(mb * (1 << 20)) // esz
        x = torch.ones(n, dtype=dt, device=dev)
        for _ in range(args.warmup):
            dist.all_reduce(x)
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            dist.all_reduce(x)
        sync()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                         device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        sec = float(t.cpu()[0]) / args.iters
        nbytes = n * esz
        algbw = nbytes / sec / 1e9
        if rank == 0:
            print(json.dumps({"bytes": nbytes, "world": world,
                              "backend": backend, "dtype": args.dtype,
                              "us": round(sec * 1e6, 1),
                              "algbw_GBs": round(algbw, 2),
                              "busbw_GBs": round(
                                  algbw * 2 * (world - 1) / max(world, 1),
                                  2)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
