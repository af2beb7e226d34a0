"""Local multi-process launcher: one data-parallel rank per GPU.

Replaces the reference's SSH/YARN node spawning and master/slave roles
(veles/launcher.py:617-660, 808-842; server.py ``--respawn`` 637-655).  Each
rank is a child process with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT set (the torch.distributed.run contract, 127.0.0.1 rendezvous).
Multi-node (``--nnodes N --node-rank R --master-addr A --master-port P``)
replaces the reference's ``-n host/devs`` SSH node list and ``-m/-l``
master/slave addresses (veles/launcher.py:199-262): every node runs this
launcher for its own GPUs, global rank = R * local ranks + local rank, and
all ranks rendezvous at A:P (RCCL over xGMI inside a node, the host network
between nodes).
Failure handling: if any rank dies, the whole group is terminated (a
collective would otherwise hang until its timeout) and, with ``respawn > 0``,
restarted from the newest ``*_current`` snapshot - the elastic-restart path
of SURVEY §5.3.
"""
from __future__ import annotations

import glob
import os
import signal
import socket
import subprocess
import sys
import time
import uuid

from veles_amd.backends import parse_device_spec

__all__ = ["spawn_ranks", "free_port", "latest_snapshot",
           "check_shared_dir", "snapshot_digest"]


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def latest_snapshot(directory):
    cands = glob.glob(os.path.join(directory, "*_current.*.pickle*"))
    cands = [c for c in cands if os.path.exists(os.path.realpath(c))]
    if not cands:
        return None
    return max(cands, key=lambda c: os.path.getmtime(os.path.realpath(c)))


def snapshot_digest(path):
    """(size, sha1) of a snapshot file: every rank of a resumed job must
    have loaded the same bytes (Launcher.initialize checks it)."""
    import hashlib
    h = hashlib.sha1()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 22), b""):
            h.update(chunk)
    return os.path.getsize(path), h.hexdigest()


def _write_atomic(path, text):
    tmp = "%s.%s.tmp" % (path, uuid.uuid4().hex)
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)


def _read(path):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def check_shared_dir(directory, nnodes, node_rank, tag, timeout=120.0,
                     poll=0.2):
    """Multi-node respawn resumes every node from ``directory``'s newest
    ``*_current`` snapshot, which only global rank 0 writes: unless the
    directory is shared by all nodes, nodes != 0 would resume from a stale
    or no snapshot and diverge (momentum, epoch, loader position).

    A challenge-response through files under ``.veles_nodes/<tag>``, with
    fresh nonces on both sides, so that files an earlier job left under the
    same tag prove nothing: node 0 publishes a random challenge; every other
    node answers it with its own random nonce; node 0 accepts once every
    node echoed THIS challenge and then publishes the accepted nonces; a
    node accepts once its own nonce is listed.  Raises ValueError when this
    does not complete within ``timeout`` seconds."""
    d = os.path.join(directory, ".veles_nodes", tag)
    os.makedirs(d, exist_ok=True)
    chal_p, done_p = os.path.join(d, "challenge"), os.path.join(d, "done")
    deadline = time.time() + timeout

    def fail(what):
        raise ValueError(
            "multi-node --respawn needs a snapshot directory shared by "
            "every node: %s shows no %s after %.0f s (mount it on all nodes "
            "or drop --respawn)" % (directory, what, timeout))

    if node_rank == 0:
        chal = uuid.uuid4().hex
        _write_atomic(chal_p, chal)
        while True:
            got = {}
            for i in range(1, nnodes):
                r = (_read(os.path.join(d, "resp%d" % i)) or "").split()
                if len(r) == 2 and r[0] == chal:
                    got[i] = r[1]
            if len(got) == nnodes - 1:
                _write_atomic(done_p, "\n".join(
                    [chal] + ["%d %s" % kv for kv in sorted(got.items())]))
                return True
            if time.time() >= deadline:
                fail("answer to this launch's challenge from node(s) %s" % (
                    ", ".join(str(i) for i in range(1, nnodes)
                              if i not in got)))
            time.sleep(poll)
    mine = uuid.uuid4().hex
    seen = None
    while True:
        chal = _read(chal_p)
        if chal and chal != seen:
            _write_atomic(os.path.join(d, "resp%d" % node_rank),
                          "%s %s" % (chal, mine))
            seen = chal
        done = (_read(done_p) or "").split("\n")
        if seen and done[0] == seen and \
                "%d %s" % (node_rank, mine) in done[1:]:
            return True
        if time.time() >= deadline:
            fail("acceptance of node %d by node 0" % node_rank)
        time.sleep(poll)


def _launch(devices, cmd, port, env_extra=None, nnodes=1, node_rank=0,
            master_addr="127.0.0.1"):
    procs = []
    n = len(devices)
    for local, dev in enumerate(devices):
        env = dict(os.environ)
        env.update({"RANK": str(node_rank * n + local),
                    "LOCAL_RANK": str(local),
                    "LOCAL_WORLD_SIZE": str(n),
                    "GROUP_RANK": str(node_rank),
                    "WORLD_SIZE": str(n * nnodes),
                    "MASTER_ADDR": master_addr,
                    "MASTER_PORT": str(port),
                    "VELES_AMD_DEVICE": str(dev)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    return procs


def _kill_all(procs):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except OSError:
                pass
    deadline = time.time() + 10
    for p in procs:
        try:
            p.wait(max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except OSError:
                pass


def spawn_ranks(spec, cmd, respawn=0, snapshot_dir=None, poll=0.5,
                shrink=False, nnodes=1, node_rank=0, master_addr=None,
                master_port=None):
    """Run ``cmd`` once per device in ``spec`` ("0-7", "0,1", "4").
    Returns the group's exit code (0 when every rank succeeded).

    ``nnodes > 1``: this call is node ``node_rank`` of a job whose nodes
    all list the same number of devices; ``master_addr``/``master_port``
    (required) name the rendezvous of global rank 0.  A failure anywhere
    ends every node's ranks (the survivors' collectives time out under
    ``--job-timeout``), so each node's launcher respawns its group and the
    job meets again at the same address.  Shrinking needs one launcher
    for the whole job and is refused here.

    ``shrink``: on a respawn, leave out the device(s) whose rank failed and
    keep the global batch by gradient accumulation - each survivor's
    optimizer step accumulates ``VELES_AMD_DP_ACCUMULATE`` = original world
    size / surviving world size micro-steps (rounded up when it does not
    divide; a warning says so)."""
    devices = parse_device_spec(spec) if isinstance(spec, str) else list(spec)
    world0 = len(devices)
    if nnodes > 1:
        if master_addr is None or master_port is None:
            raise ValueError("multi-node launch needs master_addr and "
                             "master_port")
        if not 0 <= node_rank < nnodes:
            raise ValueError("node_rank %d outside [0, %d)" %
                             (node_rank, nnodes))
        if shrink:
            raise ValueError("--respawn-shrink is single-node only")
        if respawn > 0:
            from veles_amd.utils.config import root, get
            check_shared_dir(
                snapshot_dir or get(root.common.dirs.snapshots, "."), nnodes,
                node_rank, "%s_%s" % (master_addr, master_port),
                float(os.environ.get("VELES_AMD_SHARED_DIR_TIMEOUT", 120)))
    addr = master_addr or "127.0.0.1"
    attempt = 0
    cmd = list(cmd)
    env_extra = {}
    while True:
        procs = _launch(devices, cmd, master_port or free_port(), env_extra,
                        nnodes, node_rank, addr)
        failed = None
        failed_ranks = []
        try:
            while True:
                codes = [p.poll() for p in procs]
                bad = [c for c in codes if c not in (None, 0)]
                if bad:
                    failed = bad[0]
                    failed_ranks = [i for i, c in enumerate(codes)
                                    if c not in (None, 0)]
                    break
                if all(c == 0 for c in codes):
                    return 0
                time.sleep(poll)
        except KeyboardInterrupt:
            _kill_all(procs)
            return 130
        _kill_all(procs)
        if attempt >= respawn:
            return failed
        attempt += 1
        from veles_amd.utils.config import root, get
        snap = latest_snapshot(snapshot_dir or get(root.common.dirs.snapshots,
                                                   "."))
        if snap is not None:
            cmd = [c for c in cmd]
            if "-w" in cmd:
                i = cmd.index("-w")
                del cmd[i:i + 2]
            cmd = cmd[:3] + ["-w", snap] + cmd[3:]
        if shrink and 0 < len(failed_ranks) < len(devices):
            devices = [d for i, d in enumerate(devices)
                       if i not in failed_ranks]
            acc = -(-world0 // len(devices))
            if acc * len(devices) != world0:
                print("[launch] %d ranks left of %d: global batch becomes "
                      "%d/%d of the original" % (len(devices), world0,
                                                  acc * len(devices), world0),
                      file=sys.stderr)
            env_extra = {"VELES_AMD_DP_ACCUMULATE": str(acc)}
        print("[launch] rank(s) %s failed with %s; respawn %d/%d on %s "
              "from %s" % (failed_ranks, failed, attempt, respawn, devices,
                           snap), file=sys.stderr)
