"""Parallelism: synchronous data parallelism over RCCL (xGMI), the process
launcher, HIP-graph step capture and the job farm for GA / ensembles."""


def find_dp(obj):
    """Walk unit -> workflow -> ... -> launcher and return the first ``dp``
    (DataParallel group) found, or None."""
    seen = set()
    w = obj
    while w is not None and id(w) not in seen:
        seen.add(id(w))
        d = w.__dict__ if hasattr(w, "__dict__") else {}
        dp = d.get("dp_") or d.get("dp")
        if dp is None:
            dp = getattr(type(w), "dp", None) if not isinstance(
                getattr(type(w), "dp", None), property) else None
        if dp is not None:
            return dp
        w = getattr(w, "workflow", None)
    return None
