"""Multi-GPU chunk scheduler for super-chunks.

The reference appends / decompresses a super-chunk one chunk at a time through one shared
context (blosc/schunk.c:1459-1477 blosc2_schunk_append_buffer, 1481-1530
blosc2_schunk_decompress_chunk).  Chunks are independent (each carries its own header and
bstarts; delta only references block 0 of the same chunk), so here a super-chunk is partitioned
into contiguous chunk ranges, one per rank (one process per GPU), and each rank runs ONE batch
launch of the engine over its range.  The only exchanges are distribution and collection:

  scatter_chunks     root -> ranks, raw shards (one RCCL scatter over xGMI)
  gather_compressed  ranks -> root, "gatherv": every rank packs its variable-size chunks into one
                     contiguous buffer on the device (b2h_pack_chunks), the per-chunk sizes are
                     all-gathered, and the root receives each rank's bytes straight into its slot
                     of the chunk-ordered result with grouped point-to-point receives (no padding,
                     the root receives exactly the compressed bytes).  The result carries the
                     offsets index a frame keeps (frame.c:1993).
  scatter_compressed root -> ranks, the inverse: grouped sends of each rank's contiguous span,
                     unpacked on the device into the batch layout (b2h_unpack_chunks)
  gather_chunks      ranks -> root, decompressed shards

There is no reduction anywhere, so no ring collective is involved.  Device tensors go over the
process group's backend ("nccl" = RCCL on ROCm); with the "gloo" backend (the CPU tests, or
several ranks sharing one GPU in a test) device tensors are staged through host memory.  The
per-chunk work never loops in Python: packing is one kernel (or one vectorised gather on CPU).
"""
import torch
import torch.distributed as dist


def shard_range(nchunks, world, rank):
    """Contiguous chunk range [lo, hi) of `rank` (keeps output in chunk order)."""
    return rank * nchunks // world, (rank + 1) * nchunks // world


def _max_shard(nchunks, world):
    return max(hi - lo for lo, hi in (shard_range(nchunks, world, r) for r in range(world)))


# ----------------------------------------------------------------- transport helpers ----
def _staged(group):
    """gloo moves host tensors only: device tensors are staged through host memory."""
    return dist.get_backend(group) == "gloo"


def _to_comm(t, group):
    return t.cpu() if (t.is_cuda and _staged(group)) else t


def _all_gather(t, group):
    world = dist.get_world_size(group)
    tc = _to_comm(t, group)
    outs = [torch.empty_like(tc) for _ in range(world)]
    dist.all_gather(outs, tc, group=group)
    return [o.to(t.device) for o in outs]


def _agree(ok, group):
    """All ranks agree on success (a MIN all-reduce of one flag): a rank whose chunks failed must
    not leave the collective sequence alone -- the others would block in their next collective
    until the process-group timeout.  Every rank then raises together."""
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
    if dist.get_backend(group) != "gloo":
        flag = flag.cuda()
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(flag.item())


def _p2p(sends, recvs, group):
    """Grouped point-to-point exchange: sends = [(tensor, dst)], recvs = [(tensor, src)].  Empty
    tensors are skipped (both sides know every size).  Receives land in the given tensors.

    Every rank of the group calls this (possibly with nothing to exchange: an empty shard), so
    every call starts with a barrier -- a batch_isend_irecv that is a group's first collective must
    be joined by all its ranks (torch.distributed), and a rank with nothing to send or receive makes
    no such call.  (A per-group "first call done" cache keyed by id(group) would go stale when a
    process group is destroyed and a new one reuses the id; one barrier per exchange is cheap
    next to the chunk payloads it precedes.)"""
    dist.barrier(group=group)
    ops, back = [], []
    for t, peer in sends:
        if t.numel():
            ops.append(dist.P2POp(dist.isend, _to_comm(t, group).contiguous(), dist.get_global_rank(group, peer)
                                  if group is not None else peer, group))
    for t, peer in recvs:
        if t.numel():
            tc = torch.empty(t.shape, dtype=t.dtype) if (t.is_cuda and _staged(group)) else t
            ops.append(dist.P2POp(dist.irecv, tc, dist.get_global_rank(group, peer)
                                  if group is not None else peer, group))
            back.append((tc, t))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for tc, t in back:
        if tc is not t:
            t.copy_(tc)


# ------------------------------------------------------------------ pack / unpack ----
def _index(sizes, stride):
    """(source index of every packed byte in the strided layout, offsets[n+1]) -- CPU only."""
    n = sizes.numel()
    offs = torch.zeros(n + 1, dtype=torch.int64)
    offs[1:] = torch.cumsum(sizes, 0)
    total = int(offs[-1])
    cid = torch.repeat_interleave(torch.arange(n, dtype=torch.int64), sizes)
    pos = torch.arange(total, dtype=torch.int64) - offs[cid]
    return cid * stride + pos, offs


def pack_chunks(comp, stride, cbytes, total=None):
    """Concatenate the compressed chunks of a batch (chunk i at comp[i*stride:], cbytes[i] bytes)
    into one contiguous buffer.  Returns (packed uint8, offsets int64[n+1]) on comp's device.
    `total` (the sum of cbytes, when the caller already knows it on the host) saves a host sync."""
    sizes = cbytes.to(torch.int64)
    n = sizes.numel()
    if comp.is_cuda:
        import blosc2_amd as B
        if total is None:
            total = int(sizes.sum().item())
        out = torch.empty(max(total, 1), dtype=torch.uint8, device=comp.device)
        offs = torch.empty(n + 1, dtype=torch.int64, device=comp.device)
        c32 = cbytes.to(torch.int32).contiguous()
        B.pack_chunks(comp.data_ptr(), stride, c32.data_ptr(), n, out.data_ptr(), offs.data_ptr(),
                      torch.cuda.current_stream().cuda_stream)
        return out[:total], offs
    idx, offs = _index(sizes.cpu(), stride)
    return comp[idx], offs


def unpack_chunks(packed, offsets, stride, device):
    """Inverse of pack_chunks: chunk i = packed[offsets[i]:offsets[i+1]] at out[i*stride:].
    Returns (out uint8 [n*stride], sizes int32[n])."""
    n = offsets.numel() - 1
    out = torch.zeros(max(1, n) * stride, dtype=torch.uint8, device=device)
    sizes = torch.empty(max(1, n), dtype=torch.int32, device=device)
    if n == 0:
        return out, sizes[:0]
    if out.is_cuda:
        import blosc2_amd as B
        offs = offsets.to(device=device, dtype=torch.int64).contiguous()
        src = packed.to(device)
        B.unpack_chunks(src.data_ptr(), offs.data_ptr(), n, out.data_ptr(), stride, sizes.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
        return out, sizes[:n]
    offs = offsets.cpu().to(torch.int64)
    d = offs[1:] - offs[:-1]
    idx, _ = _index(d, stride)
    out[idx] = packed.to(device)
    return out, d.to(torch.int32)


# ------------------------------------------------------------------- collectives ----
def scatter_chunks(full, chunk_nbytes, nchunks, device, root=0, group=None):
    """Distribute the raw super-chunk `full` (uint8, nchunks*chunk_nbytes, significant on root
    only) so that each rank receives its shard_range.  Returns the local uint8 shard.  Equal
    shards go in one scatter; uneven ones (nchunks % world != 0) by grouped sends."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(nchunks, world, rank)
    spans = [shard_range(nchunks, world, r) for r in range(world)]
    if len({b - a for a, b in spans}) == 1:
        recv = torch.empty((hi - lo) * chunk_nbytes, dtype=torch.uint8, device=device)
        parts = [full[a * chunk_nbytes:b * chunk_nbytes] for a, b in spans] if rank == root else None
        if _staged(group):
            rc = _to_comm(recv, group)
            dist.scatter(rc, [_to_comm(p, group).contiguous() for p in parts] if parts else None, src=root, group=group)
            recv.copy_(rc)
        else:
            dist.scatter(recv, parts, src=root, group=group)
        return recv
    recv = torch.empty((hi - lo) * chunk_nbytes, dtype=torch.uint8, device=device)
    # every rank joins one collective first: with NCCL a group's first P2P batch must include all
    # ranks, and a rank with an empty shard posts no send / receive at all
    _agree(True, group)
    if rank == root:
        recv.copy_(full[lo * chunk_nbytes:hi * chunk_nbytes])
        _p2p([(full[a * chunk_nbytes:b * chunk_nbytes], r) for r, (a, b) in enumerate(spans) if r != root], [], group)
    else:
        _p2p([], [(recv, root)], group)
    return recv


def gather_compressed(comp, stride, cbytes, nchunks, root=0, group=None, failed=False):
    """Collect every rank's compressed chunks on the root, in chunk order ("gatherv").
    Returns on the root (frame_bytes uint8, offsets int64[nchunks+1]); None elsewhere.

    The per-chunk sizes are all-gathered on the device and read back ONCE per rank: every P2P
    count, the packing total and the root's frame size come from that one copy (RCCL needs its
    counts on the host).  The same exchange carries the failure flag: a rank whose compression
    failed (`failed`, or a chunk of size <= 0) sends -1 sizes, and every rank raises together
    after the read-back -- no separate agreement round."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = comp.device
    mx = _max_shard(nchunks, world)
    spans = [shard_range(nchunks, world, q) for q in range(world)]
    sz = torch.zeros(mx + 1, dtype=torch.int64, device=dev)
    sz[:cbytes.numel()] = cbytes.to(torch.int64)
    if failed:
        sz[:cbytes.numel()] = -1
    sz[mx] = -1 if failed else 0
    all_sz = torch.stack(_all_gather(sz, group)).cpu()   # the one host sync
    lens = torch.cat([all_sz[r, :b - a] for r, (a, b) in enumerate(spans)])
    bad = [r for r, (a, b) in enumerate(spans) if int(all_sz[r, mx]) < 0 or bool((all_sz[r, :b - a] <= 0).any())]
    if bad:
        raise RuntimeError(f"rank {rank}: compression failed on rank(s) {bad}")
    host_off = [0] + torch.cumsum(lens, 0).tolist()
    a, b = spans[rank]
    packed, _ = pack_chunks(comp, stride, cbytes, total=host_off[b] - host_off[a])
    if rank != root:
        _p2p([(packed, root)], [], group)
        return None
    offsets = torch.tensor(host_off, dtype=torch.int64).to(dev, non_blocking=True)
    frame = torch.empty(int(host_off[-1]), dtype=torch.uint8, device=dev)
    recvs = []
    for r, (a, b) in enumerate(spans):
        piece = frame[host_off[a]:host_off[b]]
        if r == root:
            piece.copy_(packed)
        else:
            recvs.append((piece, r))
    _p2p([], recvs, group)
    return frame, offsets


def scatter_compressed(frame, offsets, nchunks, stride, device, root=0, group=None):
    """Inverse of gather_compressed: each rank receives its chunk range laid out at `stride`
    (ready for b2h_decompress_batch) plus the per-chunk sizes (int32)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(nchunks, world, rank)
    # every rank learns the offsets index (nchunks + 1 int64, a broadcast of a few KiB)
    off = offsets.to(device=device, dtype=torch.int64) if rank == root else \
        torch.empty(nchunks + 1, dtype=torch.int64, device=device)
    oc = _to_comm(off, group)
    dist.broadcast(oc, src=root, group=group)
    if oc is not off:
        off.copy_(oc)
    host_off = off.cpu().tolist()
    span = torch.empty(int(host_off[hi] - host_off[lo]), dtype=torch.uint8, device=device)
    if rank == root:
        span.copy_(frame[int(host_off[lo]):int(host_off[hi])].to(device))
        sends = []
        for r in range(world):
            a, b = shard_range(nchunks, world, r)
            if r != root:
                sends.append((frame[int(host_off[a]):int(host_off[b])].to(device), r))
        _p2p(sends, [], group)
    else:
        _p2p([], [(span, root)], group)
    local_off = off[lo:hi + 1] - off[lo]
    return unpack_chunks(span, local_off, stride, device)


def gather_chunks(local, chunk_nbytes, nchunks, root=0, group=None):
    """Collect the decompressed shards on the root in chunk order (inverse of scatter_chunks)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if rank != root:
        _p2p([(local, root)], [], group)
        return None
    out = torch.empty(nchunks * chunk_nbytes, dtype=torch.uint8, device=local.device)
    recvs = []
    for r in range(world):
        a, b = shard_range(nchunks, world, r)
        piece = out[a * chunk_nbytes:b * chunk_nbytes]
        if r == root:
            piece.copy_(local)
        else:
            recvs.append((piece, r))
    _p2p([], recvs, group)
    return out


# ------------------------------------------------------------- engine + pipelines ----
def device_engine(cparams):
    """(compress_batch, decompress_batch) callables over the MI355X engine on torch's current
    stream, in the signatures compress_schunk / decompress_schunk take."""
    import blosc2_amd as B
    cp = B.cparams(**cparams)

    def comp(_, src, chunk_nbytes, n, out, stride, cap, cbytes):
        B.compress_batch(cp, src.data_ptr(), chunk_nbytes, n, chunk_nbytes, out.data_ptr(), stride, cap,
                         cbytes.data_ptr(), torch.cuda.current_stream().cuda_stream)

    def decomp(comp_buf, stride, cbytes, n, out, chunk_nbytes):
        status = torch.empty(n, dtype=torch.int32, device=out.device)
        B.decompress_batch(comp_buf.data_ptr(), stride, cbytes.data_ptr(), n, out.data_ptr(), chunk_nbytes,
                           chunk_nbytes, status.data_ptr(), torch.cuda.current_stream().cuda_stream)
        return status

    return comp, decomp


def compress_schunk(full, chunk_nbytes, nchunks, cparams, device, compress_batch, root=0, group=None):
    """Distributed super-chunk compression: scatter raw shards, compress each rank's range with
    `compress_batch(cparams, src_u8, chunk_nbytes, n, comp_u8, stride, cap, cbytes_i32)` (the
    device batch engine on GPUs), gather the compressed chunks in order on the root.
    Returns (frame, offsets) on the root, None elsewhere."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(nchunks, world, rank)
    local = scatter_chunks(full, chunk_nbytes, nchunks, device, root, group)
    cap = chunk_nbytes + 32
    stride = (cap + 255) // 256 * 256
    n = hi - lo
    comp = torch.empty(max(1, n) * stride, dtype=torch.uint8, device=device)
    cbytes = torch.zeros(max(1, n), dtype=torch.int32, device=device)
    failed = False
    if n:
        try:
            compress_batch(cparams, local, chunk_nbytes, n, comp, stride, cap, cbytes)
        except RuntimeError:
            failed = True
    # a chunk of size <= 0 (did not fit: cannot happen at cap = nbytes + 32) or a failed launch is
    # seen by every rank in the gather's size exchange, which then raises everywhere together
    return gather_compressed(comp, stride, cbytes[:n], nchunks, root, group, failed=failed)


def decompress_schunk(frame, offsets, chunk_nbytes, nchunks, device, decompress_batch, root=0, group=None):
    """Inverse of compress_schunk: returns the raw super-chunk on the root, None elsewhere."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(nchunks, world, rank)
    cap = chunk_nbytes + 32
    stride = (cap + 255) // 256 * 256
    comp, cbytes = scatter_compressed(frame, offsets, nchunks, stride, device, root, group)
    n = hi - lo
    out = torch.empty(max(1, n) * chunk_nbytes, dtype=torch.uint8, device=device)
    err = None
    if n:
        try:
            status = decompress_batch(comp, stride, cbytes, n, out, chunk_nbytes)
            if status is not None and not bool((status == chunk_nbytes).all()):
                err = f"rank {rank}: decompression status {status.min().item()}"
        except RuntimeError as e:
            err = f"rank {rank}: {e}"
    if not _agree(err is None, group):
        raise RuntimeError(err or f"rank {rank}: another rank failed to decompress its chunks")
    return gather_chunks(out[:n * chunk_nbytes], chunk_nbytes, nchunks, root, group)
