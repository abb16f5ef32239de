"""Multi-GPU chunk scheduler for super-chunks.

The reference appends / decompresses a super-chunk one chunk at a time through one shared
context (blosc/schunk.c:1459-1477 blosc2_schunk_append_buffer, 1481-1530
blosc2_schunk_decompress_chunk).  Chunks are independent (each carries its own header and
bstarts; delta only references block 0 of the same chunk), so here a super-chunk is partitioned
into contiguous chunk ranges, one per rank (one process per GPU), and each rank runs the batch
engine on its range.  The only exchanges are distribution and collection:

  scatter_chunks     root -> ranks, equal-size raw shards (RCCL scatter over xGMI)
  gather_compressed  ranks -> root, variable-size compressed chunks + the per-chunk sizes,
                     assembled on the root into chunk order with an offsets index (the
                     information a frame's chunk-offsets index holds, frame.c:1993)
  scatter_compressed root -> ranks, the inverse for decompression
  gather_chunks      ranks -> root, decompressed shards

There is no reduction anywhere, so no ring collective is involved.  Every function takes the
process group's backend as given ("nccl" = RCCL on ROCm for device tensors, "gloo" for the CPU
tests) and works on whatever device the tensors live on.
"""
import torch
import torch.distributed as dist


def shard_range(nchunks, world, rank):
    """Contiguous chunk range [lo, hi) of `rank` (keeps output in chunk order)."""
    return rank * nchunks // world, (rank + 1) * nchunks // world


def _max_shard(nchunks, world):
    return max(hi - lo for lo, hi in (shard_range(nchunks, world, r) for r in range(world)))


def scatter_chunks(full, chunk_nbytes, nchunks, device, root=0, group=None):
    """Distribute the raw super-chunk `full` (uint8, nchunks*chunk_nbytes, significant on root
    only) so that each rank receives its shard_range.  Returns the local uint8 shard."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(nchunks, world, rank)
    cap = _max_shard(nchunks, world) * chunk_nbytes
    recv = torch.empty(cap, dtype=torch.uint8, device=device)
    parts = None
    if rank == root:
        parts = []
        for r in range(world):
            a, b = shard_range(nchunks, world, r)
            p = full[a * chunk_nbytes:b * chunk_nbytes]
            if p.numel() < cap:                      # equal-size scatter: pad the short shards
                p = torch.cat([p, torch.zeros(cap - p.numel(), dtype=torch.uint8, device=device)])
            parts.append(p.contiguous())
    dist.scatter(recv, parts, src=root, group=group)
    return recv[:(hi - lo) * chunk_nbytes]


def pack_chunks(comp, stride, cbytes):
    """Concatenate the compressed chunks of a batch (chunk i at comp[i*stride:], cbytes[i] bytes)
    into one contiguous buffer.  Returns (packed uint8, sizes int64 on the same device)."""
    sizes = cbytes.to(torch.int64)
    host = sizes.cpu().tolist()
    total = int(sum(host))
    out = torch.empty(total, dtype=torch.uint8, device=comp.device)
    o = 0
    for i, n in enumerate(host):
        out[o:o + n] = comp[i * stride:i * stride + n]
        o += n
    return out, sizes


def gather_compressed(comp, stride, cbytes, nchunks, root=0, group=None):
    """Collect every rank's compressed chunks on the root, in chunk order.
    Returns on the root (frame_bytes uint8, offsets int64[nchunks+1]); None elsewhere."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = comp.device
    packed, sizes = pack_chunks(comp, stride, cbytes)
    mx = _max_shard(nchunks, world)
    # per-chunk sizes of every rank (fixed count: pad to the largest shard)
    sz = torch.zeros(mx, dtype=torch.int64, device=dev)
    sz[:sizes.numel()] = sizes
    all_sz = [torch.zeros(mx, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(all_sz, sz, group=group)
    totals = [int(t.sum().item()) for t in all_sz]
    cap = max(totals) if totals else 0
    buf = torch.zeros(cap, dtype=torch.uint8, device=dev)
    buf[:packed.numel()] = packed
    bufs = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == root else None
    dist.gather(buf, bufs, dst=root, group=group)
    if rank != root:
        return None
    pieces, lens = [], []
    for r in range(world):
        lo, hi = shard_range(nchunks, world, r)
        pieces.append(bufs[r][:totals[r]])
        lens.append(all_sz[r][:hi - lo])
    frame = torch.cat(pieces)
    offsets = torch.zeros(nchunks + 1, dtype=torch.int64, device=dev)
    offsets[1:] = torch.cumsum(torch.cat(lens), 0)
    return frame, offsets


def scatter_compressed(frame, offsets, nchunks, stride, device, root=0, group=None):
    """Inverse of gather_compressed: each rank receives its chunk range laid out at `stride`
    (ready for b2h_decompress_batch) plus the per-chunk sizes (int32)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(nchunks, world, rank)
    mx = _max_shard(nchunks, world)
    # sizes first (fixed count), then each shard's packed bytes padded to the largest
    sizes = torch.zeros(mx, dtype=torch.int64, device=device)
    parts_sz, spans = None, None
    if rank == root:
        off = offsets.to(device)
        d = off[1:] - off[:-1]
        parts_sz, spans = [], []
        for r in range(world):
            a, b = shard_range(nchunks, world, r)
            p = torch.zeros(mx, dtype=torch.int64, device=device)
            p[:b - a] = d[a:b]
            parts_sz.append(p)
            spans.append(int(off[b] - off[a]))
        span_t = torch.tensor([max(spans)], dtype=torch.int64, device=device)
    else:
        span_t = torch.zeros(1, dtype=torch.int64, device=device)
    dist.scatter(sizes, parts_sz, src=root, group=group)
    dist.broadcast(span_t, src=root, group=group)
    cap = int(span_t.item())
    recv = torch.empty(cap, dtype=torch.uint8, device=device)
    parts = None
    if rank == root:
        parts = []
        for r in range(world):
            a, b = shard_range(nchunks, world, r)
            p = frame[int(offsets[a]):int(offsets[b])].to(device)
            if p.numel() < cap:
                p = torch.cat([p, torch.zeros(cap - p.numel(), dtype=torch.uint8, device=device)])
            parts.append(p.contiguous())
    dist.scatter(recv, parts, src=root, group=group)
    n = hi - lo
    host = sizes[:n].cpu().tolist()
    comp = torch.zeros(n * stride, dtype=torch.uint8, device=device)
    o = 0
    for i, c in enumerate(host):
        comp[i * stride:i * stride + c] = recv[o:o + c]
        o += c
    return comp, sizes[:n].to(torch.int32)


def gather_chunks(local, chunk_nbytes, nchunks, root=0, group=None):
    """Collect the decompressed shards on the root in chunk order (inverse of scatter_chunks)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    cap = _max_shard(nchunks, world) * chunk_nbytes
    buf = torch.zeros(cap, dtype=torch.uint8, device=local.device)
    buf[:local.numel()] = local
    bufs = [torch.empty(cap, dtype=torch.uint8, device=local.device) for _ in range(world)] \
        if rank == root else None
    dist.gather(buf, bufs, dst=root, group=group)
    if rank != root:
        return None
    out = []
    for r in range(world):
        a, b = shard_range(nchunks, world, r)
        out.append(bufs[r][:(b - a) * chunk_nbytes])
    return torch.cat(out)


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
    if n:
        compress_batch(cparams, local, chunk_nbytes, n, comp, stride, cap, cbytes)
    return gather_compressed(comp, stride, cbytes[:n], nchunks, root, group)


def decompress_schunk(frame, offsets, chunk_nbytes, nchunks, device, decompress_batch, root=0, group=None):
    """Inverse of compress_schunk: returns the raw super-chunk on the root, None elsewhere."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(nchunks, world, rank)
    cap = chunk_nbytes + 32
    stride = (cap + 255) // 256 * 256
    comp, cbytes = scatter_compressed(frame, offsets, nchunks, stride, device, root, group)
    n = hi - lo
    out = torch.empty(max(1, n) * chunk_nbytes, dtype=torch.uint8, device=device)
    if n:
        decompress_batch(comp, stride, cbytes, n, out, chunk_nbytes)
    return gather_chunks(out[:n * chunk_nbytes], chunk_nbytes, nchunks, root, group)
