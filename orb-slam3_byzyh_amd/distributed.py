"""Frame-sharded batch extraction across GPUs with an all-gather of the features (C4).

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm; "gloo" on CPU for tests).
Frames are independent units.  Rank r extracts frames [r*B, (r+1)*B) of the global batch into
fixed-capacity blocks, then a single all-gather over xGMI gives every rank the features of all
frames: descriptors [W*B, cap, 32] u8, keypoints [W*B, cap, 7] (cv::KeyPoint layout) and counts
[W*B, 2].  Cross-frame matching then runs locally against the gathered set: each rank matches its
own frames against their predecessors in the global batch (knn2, src/ORBmatcher.cc
DescriptorDistance; one orb_hamming_knn2_frames_device launch for all of the rank's frames).

The all-gather is the only data-path collective.  It is issued asynchronously on RCCL's stream
and double-buffered, so step i's exchange overlaps step i+1's extraction.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous frame range of `rank` (the first n_total % world ranks take one extra frame)."""
    base, extra = divmod(n_total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


class FeatureBlocks:
    """Fixed-capacity per-frame feature blocks (the extractor's device output layout)."""

    def __init__(self, frames: int, cap: int, device, count: int = 1):
        self.frames, self.cap = frames, cap
        self.kps = torch.empty((count, frames, cap, 7), dtype=torch.float32, device=device)
        self.desc = torch.empty((count, frames, cap, 32), dtype=torch.uint8, device=device)
        self.counts = torch.empty((count, frames, 2), dtype=torch.int32, device=device)

    def view(self, i: int = 0):
        return self.kps[i], self.desc[i], self.counts[i]


def all_gather_features(kps, desc, counts, group=None, async_op: bool = False):
    """All-gather one rank's feature blocks; returns (gathered kps, desc, counts[, work handles]).
    With the gloo backend (CPU tests, single-GPU rehearsals) device tensors are staged on the host."""
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo" and kps.is_cuda:
        out = all_gather_features(kps.cpu(), desc.cpu(), counts.cpu(), group, False)
        out = tuple(t.to(kps.device) for t in out)
        return out + ([],) if async_op else out
    g_kps = torch.empty((world * kps.shape[0],) + tuple(kps.shape[1:]), dtype=kps.dtype, device=kps.device)
    g_desc = torch.empty((world * desc.shape[0],) + tuple(desc.shape[1:]), dtype=desc.dtype, device=desc.device)
    g_cnt = torch.empty((world * counts.shape[0],) + tuple(counts.shape[1:]), dtype=counts.dtype,
                        device=counts.device)
    works = [dist.all_gather_into_tensor(g_desc, desc.contiguous(), group=group, async_op=async_op),
             dist.all_gather_into_tensor(g_kps, kps.contiguous(), group=group, async_op=async_op),
             dist.all_gather_into_tensor(g_cnt, counts.contiguous(), group=group, async_op=async_op)]
    if async_op:
        return g_kps, g_desc, g_cnt, works
    return g_kps, g_desc, g_cnt


class ShardedExtractor:
    """ORB extraction of a global frame batch sharded over the ranks of a process group."""

    def __init__(self, extractor, frames_per_rank: int, cap: int | None = None, group=None, match: bool = False):
        """`extractor`: one ORBextractor, or a list of them used in turn (batches in flight on their
        own streams: pass step i's stream as stream i % len).  match: after each all-gather, knn2 of
        this rank's frames against their predecessors in the gathered blocks (self.matches)."""
        self.exs = list(extractor) if isinstance(extractor, (list, tuple)) else [extractor]
        self.ex = self.exs[0]
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.frames = frames_per_rank
        self.cap = cap or (self.ex.nfeatures + 16 * self.ex.nlevels)
        dev = torch.device("cuda", torch.cuda.current_device())
        # len(exs) + 1 blocks: step i + len + 1 reuses step i's block on the stream of step i + 1, which
        # waited for step i's all-gather (finish) before anything it enqueues later
        self.nbuf = len(self.exs) + 1
        self.local = FeatureBlocks(frames_per_rank, self.cap, dev, count=self.nbuf)
        self._i = 0
        self._pending = None
        self.match = match
        # (idx, best, second) [frames_per_rank, cap] of the latest gathered step: inside step() that is
        # the previous step's gather, after finish() the last one.  The tensors cycle through nbuf
        # buffers, so a result is overwritten nbuf steps later: copy it to keep it.
        self.matches = None
        if match:
            first = self.rank * frames_per_rank  # equal shards: global frame f sits at row f of the gather
            self.pairs = frame_pairs(first, frames_per_rank, self.world * frames_per_rank).to(dev)
            self._mbuf = [tuple(torch.empty((frames_per_rank, self.cap), dtype=torch.int32, device=dev)
                                for _ in range(3)) for _ in range(self.nbuf)]

    def step(self, images, vLappingArea=(0, 0), stream=None):
        """Extract this rank's frames (uint8 [B, H, W] on the GPU) and start the all-gather.
        Returns the previous step's gathered blocks (or None on the first call)."""
        buf = self._i % self.nbuf
        out = self.local.view(buf)
        self.exs[self._i % len(self.exs)].extract_batch_device(images, vLappingArea, cap=self.cap, out=out,
                                                               stream=stream)
        prev = self._wait(stream)
        self._match(prev, stream)
        # RCCL orders a collective after torch's CURRENT stream only: issue it with the extraction
        # stream current, so it cannot read the blocks before the extraction has written them
        with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            self._pending = all_gather_features(*out, group=self.group, async_op=True)
        self._i += 1
        return prev

    def _match(self, gathered, stream):
        if self.match and gathered is not None:  # the gather of step self._i - 1
            self.matches = match_gathered(gathered[1], gathered[2], self.pairs, stream=stream,
                                          out=self._mbuf[(self._i - 1) % self.nbuf])

    def finish(self, stream=None):
        """Make `stream` (default: the current stream) wait for the in-flight all-gather and return
        its (kps, desc, counts); with match=True the last step's gather is matched too (self.matches)."""
        gathered = self._wait(stream)
        self._match(gathered, stream)
        return gathered

    def _wait(self, stream=None):
        if self._pending is None:
            return None
        g_kps, g_desc, g_cnt, works = self._pending
        with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            for w in works:
                w.wait()
            # the gathered blocks were allocated while another step's stream was current; tell the
            # caching allocator that `stream` uses them too, so their memory is not handed to a later
            # all-gather (ordered only after its own stream) before this stream has read them
            consumer = torch.cuda.current_stream()
            for t in (g_kps, g_desc, g_cnt):
                if t.is_cuda:
                    t.record_stream(consumer)
        self._pending = None
        return g_kps, g_desc, g_cnt


def _knn2_device(query, train):
    from .matcher import ORBmatcher
    return ORBmatcher.knn2_device(query, train)


def distributed_knn2(query, train, group=None, local_fn=None):
    """Best / second-best Hamming match of every query row against the whole train set, with the
    query rows split over the ranks (Hamming matching): rank r matches rows
    [r * P, (r + 1) * P), P = ceil(n_query / world), locally (knn2 kernel, orb_hamming_knn2_device) and one all-gather
    of the per-query results (best index, best distance, second distance: 12 B per query) gives every
    rank the full answer.  Every rank passes the same query and train tensors (uint8 [n, 32]; e.g. a
    frame's descriptors and the all-gathered descriptors of the other frames).  The result equals
    the single-device knn2 exactly: each query's scan is unchanged, only the rows are distributed.
    `local_fn(query_rows, train) -> (idx, best, second)` replaces the device kernel (CPU tests)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = query.shape[0]
    fn = local_fn or _knn2_device
    if world == 1:
        return fn(query, train)
    per = (n + world - 1) // world  # equal blocks for all_gather_into_tensor; the last one is padded
    b0, b1 = min(n, rank * per), min(n, (rank + 1) * per)
    idx, d1, d2 = fn(query[b0:b1], train)
    block = torch.full((3, per), -1, dtype=torch.int32, device=query.device)
    if b1 > b0:
        block[0, : b1 - b0] = idx
        block[1, : b1 - b0] = d1
        block[2, : b1 - b0] = d2
    gathered = torch.empty((world * 3, per), dtype=torch.int32, device=query.device)
    if dist.get_backend(group) == "gloo" and block.is_cuda:
        host = torch.empty((world * 3, per), dtype=torch.int32)
        dist.all_gather_into_tensor(host, block.cpu(), group=group)
        gathered.copy_(host)
    else:
        dist.all_gather_into_tensor(gathered, block, group=group)
    flat = gathered.view(world, 3, per).permute(1, 0, 2).reshape(3, world * per)[:, :n]
    return flat[0].contiguous(), flat[1].contiguous(), flat[2].contiguous()


def frame_pairs(first: int, count: int, n_total: int) -> torch.Tensor:
    """(query frame, train frame) = (f, f - 1 mod n_total) for frames f in [first, first + count): each
    frame against its predecessor in the global batch (frame 0 against the last), as tracking matches a
    frame against the previous one.  int32 [count, 2] (CPU)."""
    f = torch.arange(first, first + count, dtype=torch.int32)
    return torch.stack([f, (f - 1) % n_total], 1).to(torch.int32)


def match_gathered(g_desc, g_cnt, pairs, local_fn=None, stream=None, out=None):
    """knn2 of each pair's query frame against its train frame in gathered feature blocks (desc
    [F, cap, 32], counts [F, 2], pairs int32 [P, 2]): one device launch (orb_hamming_knn2_frames_device).
    `local_fn(query_rows, train_rows) -> (idx, best, second)` replaces it pair by pair (CPU tests).
    Returns (idx, best, second), int32 [P, cap]; rows beyond a query frame's count hold (-1, 257, 257)."""
    if local_fn is None:
        from .matcher import ORBmatcher
        return ORBmatcher.knn2_frames_device(g_desc, g_cnt, pairs, stream=stream, out=out)
    n_pairs, cap = pairs.shape[0], g_desc.shape[1]
    res = tuple(torch.full((n_pairs, cap), v, dtype=torch.int32) for v in (-1, 257, 257))
    for p, (qf, tf) in enumerate(pairs.tolist()):
        nq, nt = int(g_cnt[qf, 0]), int(g_cnt[tf, 0])
        got = local_fn(g_desc[qf, :nq].cpu(), g_desc[tf, :nt].cpu())
        for k in range(3):
            res[k][p, :nq] = got[k]
    return res


def frame_descriptors(g_desc, g_cnt, frame: int):
    """Descriptors of global frame `frame` from the gathered blocks (a view, count rows)."""
    n = int(g_cnt[frame, 0])
    return g_desc[frame, :n]
