"""Multi-GPU plumbing for the classification path.

Packets are independent, so a batch shards across ranks with no data-path
collective: every rank holds the same compiled tables (replicated, same
seeds) and classifies its own contiguous slice.  The only exchange is the
per-rule hit counters, summed once per batch.  The three counter spaces of
a classifier (ACL, route, group; include/vclassify.h VC_COUNTERS_*) are
packed into ONE int64 bucket so a batch costs a single all-reduce: on
xGMI a ring all-reduce is per-link bound and the ~10 MB bucket is large
enough to stream at link rate, where three small calls would each pay the
ring's latency.

The reference has no counterpart: vproxy is one JVM per host, and its
SecurityGroup / RouteTable / Upstream keep no hit counters.  The counters are
the north-star's "per-rule hit counters" (BASELINE.json).
"""
import ctypes as C

__all__ = ["shard", "HitCounterBucket", "check_replicated"]


def shard(n, rank, world):
    """Contiguous slice [lo, hi) of an n-item batch owned by `rank`.
    The first n % world ranks take one extra item, so slices differ by at
    most one and cover 0..n exactly once."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank %d of %d" % (rank, world))
    q, r = divmod(int(n), world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


_hip = None


def _hip_memcpy_d2d(dst_ptr, src_ptr, nbytes, stream):
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int,
                                        C.c_void_p]
    rc = _hip.hipMemcpyAsync(C.c_void_p(dst_ptr), C.c_void_p(src_ptr), nbytes, 3,  # D2D
                             C.c_void_p(stream))
    if rc != 0:
        raise RuntimeError("hipMemcpyAsync failed: %d" % rc)


class HitCounterBucket:
    """One flat int64 tensor holding several counter spaces back to back.

    sizes:   number of uint64 counters of each space (e.g. the `n` returned
             by Classifier.counters_device for ACL, ROUTE, GROUP)
    device:  torch device of the bucket (cuda:k for RCCL, cpu for gloo)

    fill(i, src) copies space i in, either from a tensor or from a raw device
    pointer of the library's counter array (a device-to-device copy on the
    current stream); reduce() sums the bucket over the process group;
    views[i] are the per-space slices of the result.
    Counts are uint64 in the library and int64 here: same bits, and no
    realistic count reaches 2^63.
    """

    def __init__(self, sizes, device):
        import torch
        self.sizes = [int(s) for s in sizes]
        self.offsets = []
        o = 0
        for s in self.sizes:
            self.offsets.append(o)
            o += s
        self.bucket = torch.zeros(max(1, o), dtype=torch.int64, device=device)
        self.views = [self.bucket[a:a + s] for a, s in zip(self.offsets, self.sizes)]

    def fill(self, i, src):
        import torch
        if isinstance(src, torch.Tensor):
            if src.numel() != self.sizes[i]:
                raise ValueError("space %d: %d counters, bucket slot %d" %
                                 (i, src.numel(), self.sizes[i]))
            self.views[i].copy_(src.view(torch.int64) if src.dtype == torch.uint64 else src)
        else:
            ptr, n = src
            if n != self.sizes[i]:
                raise ValueError("space %d: %d counters, bucket slot %d" % (i, n, self.sizes[i]))
            if n:
                _hip_memcpy_d2d(self.views[i].data_ptr(), ptr, n * 8,
                                torch.cuda.current_stream().cuda_stream)

    def reduce(self, group=None):
        """Sum over ranks in place (one collective for all spaces)."""
        import torch.distributed as dist
        dist.all_reduce(self.bucket, op=dist.ReduceOp.SUM, group=group)
        return self.views


def check_replicated(digests, group=None):
    """Summed hit counters mean something only if every rank classified
    against the same tables.  `digests`: this rank's table digests
    (Classifier.table_digest per counter space, or the host-only
    vproxy_amd.digest_* forms).  All-gathers them over the process group
    (one small collective, before any batch) and raises if any rank
    compiled a different image.  Returns the list of every rank's digests."""
    import torch
    import torch.distributed as dist
    mine = torch.tensor([d - (1 << 64) if d >= 1 << 63 else d for d in digests],
                        dtype=torch.int64)
    backend = dist.get_backend(group)
    if backend == "nccl":
        mine = mine.cuda()
    got = [torch.zeros_like(mine) for _ in range(dist.get_world_size(group))]
    dist.all_gather(got, mine, group=group)
    rows = [[int(x) & ((1 << 64) - 1) for x in g.cpu().tolist()] for g in got]
    bad = [r for r, row in enumerate(rows) if row != rows[0]]
    if bad:
        raise RuntimeError("ranks %s compiled different tables than rank 0: %s" % (bad, rows))
    return rows
