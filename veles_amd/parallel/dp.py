"""Synchronous data parallelism over RCCL (``torch.distributed`` backend
"nccl" is RCCL on ROCm), one process per MI355X.

Replaces the reference's asynchronous ZeroMQ master/slave parameter exchange
(veles/server.py, veles/client.py, veles/workflow.py:456-548; SURVEY §2.6,
§2.7, Appendix D):

* weights are broadcast once from rank 0 (``broadcast_``);
* gradients are all-reduced (SUM; the loss is already averaged over the
  GLOBAL batch) in contiguous fp32 buckets of the flat gradient buffer,
  launched asynchronously the moment a bucket's last layer has enqueued its
  gradient kernels - RCCL's stream waits on the compute stream at that point,
  so the reduction of the classifier layers overlaps the convolution backward;
* the fused optimizer step waits on the bucket handles (stream-level waits,
  no host synchronisation);
* class-end metrics are summed so every rank takes identical decisions.

Bucket size: xGMI is point-to-point (7 links x ~153 GB/s per MI355X).  RCCL's
ring/tree channels stripe one collective over the links; buckets of
>= 32 MB keep each ring step bandwidth-bound (latency ~10-20 us per step)
while still leaving several buckets to overlap (docs/PARALLEL.md).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

__all__ = ["DataParallel", "init_from_env"]


class DataParallel(object):
    def __init__(self, backend=None, timeout_s=600, device=None):
        self.world_size = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        self.backend = backend
        self.device = device
        # VELES_AMD_DP_SOLO_COLLECTIVES=1 at world size 1: a one-rank process
        # group that runs the whole multi-rank gradient path (bucketed
        # all-reduces, per-bucket updates, eager steps) - the RCCL stream
        # semantics of that path measured on a single GPU
        self.solo = self.world_size == 1 and os.environ.get(
            "VELES_AMD_DP_SOLO_COLLECTIVES", "0") == "1"
        if (self.world_size > 1 or self.solo) and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29511")
            kw = {}
            if backend == "nccl":
                torch.cuda.set_device(self.local_rank)
                kw["device_id"] = torch.device("cuda", self.local_rank)
            dist.init_process_group(
                backend, rank=self.rank, world_size=self.world_size,
                timeout=datetime.timedelta(seconds=timeout_s), **kw)
        self.group = dist.group.WORLD if self.multi else None

    @property
    def is_master(self):
        return self.rank == 0

    @property
    def multi(self):
        """True when gradients go through collectives (several ranks, or a
        solo process group)."""
        return self.world_size > 1 or self.solo

    @property
    def host_blocking_wait(self):
        """gloo's ``Work.wait()`` blocks the host until the collective is
        done; RCCL's only makes the current stream wait on it."""
        return self.backend != "nccl"

    def all_reduce_async(self, tensor):
        if not self.multi:
            return _Done()
        return dist.all_reduce(tensor, op=dist.ReduceOp.SUM, async_op=True)

    def all_reduce_sum(self, tensor):
        if self.world_size > 1:
            t = tensor
            if self.backend == "nccl" and not t.is_cuda:
                t = t.cuda()
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            if t is not tensor:
                tensor.copy_(t.cpu())
        return tensor

    def all_reduce_max(self, tensor):
        if self.world_size > 1:
            dist.all_reduce(tensor, op=dist.ReduceOp.MAX)
        return tensor

    def agree(self, flag, src=0):
        """Rank ``src``'s boolean, on every rank (one tiny broadcast): for
        decisions taken from a local clock that must be collective."""
        if self.world_size <= 1:
            return bool(flag)
        import torch
        dev = torch.device("cuda", torch.cuda.current_device()) \
            if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
        dist.broadcast(t, src)
        return bool(t.item())

    def broadcast_(self, tensor, src=0):
        if self.world_size > 1:
            dist.broadcast(tensor, src)
        return tensor

    def barrier(self):
        if self.world_size > 1:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    def all_gather_object(self, obj):
        if self.world_size <= 1:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj)
        return out

    def shutdown(self):
        """Destroy the process group while the interpreter is fully alive.

        ``self.group`` held the WORLD ProcessGroup object: with it alive,
        destroy_process_group() did not destroy the gloo group, whose
        worker threads then outlived ``main``.  A worker that was still
        releasing its last work item at interpreter exit (the item's tensors
        carry Python objects, so the release takes the GIL) hit the
        finalizing interpreter, which ends such a thread with pthread_exit;
        the forced unwind through the C++ thread function aborted the rank
        with "terminate called without an active exception" (backtrace:
        ProcessGroupGloo::runLoop -> TensorImpl::decref_pyobject ->
        PyEval_AcquireThread -> pthread_exit; about 1 run in 40 of
        test_dp_snapshotter_decision_is_collective under load,
        docs/PARALLEL.md).  Dropping the reference and collecting lets the
        group's destructor join its threads here instead."""
        from veles_amd.ops import fp8
        fp8.release_dp(self)
        self.group = None
        if self.multi and dist.is_initialized():
            dist.destroy_process_group()
        import gc
        gc.collect()

    def __getstate__(self):
        raise TypeError("DataParallel groups are not picklable")


class _Done(object):
    def wait(self):
        return True


def init_from_env(**kwargs):
    return DataParallel(**kwargs)
