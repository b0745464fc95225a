"""parallel.py — record-sharded XDR encode/decode across GPUs (one process per GPU).

Records are independent (no cross-record state in org.dcache.oncrpc4j.xdr.Xdr;
an XdrAble encodes into the stream in order), so a batch of N
records shards into contiguous record ranges, rank r owning
[r*N/G, (r+1)*N/G).  Encode and decode need no collective.  Reassembling
one contiguous XDR stream (BASELINE configs[4]) is the only exchange, and it
moves exactly the shard bytes:

* the shard byte counts are all-gathered (G x u64) and prefix-summed: rank r's
  shard lands at sum(sizes[:r]);
* equal sizes (fixed-size records): one rank-ordered all-gather straight into
  the output (RCCL `all_gather_into_tensor` over xGMI) is the single-GPU
  stream;
* unequal sizes (variable-size records): RCCL has no all-gather-v, so every
  rank sends its shard to every peer and receives each peer's shard into its
  exact slice, as one grouped batch of send/recv (`batch_isend_irecv`, which
  the nccl backend issues inside one ncclGroupStart/End: the G-1 transfers
  run concurrently over the point-to-point xGMI links, no padding moves).
  Record offsets are rebased by the shard's prefix and exchanged the same way.

The collectives run on the process group's backend: nccl (RCCL) on MI355X,
gloo in the CPU tests.  The per-shard codec is passed in (the HIP engine in
production), so this module holds only the sharding and exchange logic.
"""
import torch
import torch.distributed as dist


def shard_range(n, world, rank):
    """Contiguous record range [lo, hi) of `rank` out of `world`."""
    return (n * rank) // world, (n * (rank + 1)) // world


def _coll_device(group=None):
    """Device the group's collectives take tensors on (RCCL: the current GPU)."""
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
        else torch.device("cpu")


def all_gather_ints(x, group=None):
    """All-gather one Python int per rank -> list in rank order."""
    world = dist.get_world_size(group)
    dev = _coll_device(group)
    mine = torch.tensor([int(x)], dtype=torch.int64, device=dev)
    out = torch.zeros(world, dtype=torch.int64, device=dev)
    if dev.type == "cuda":
        dist.all_gather_into_tensor(out, mine, group=group)
    else:
        parts = list(out.split(1))
        dist.all_gather(parts, mine, group=group)
        out = torch.cat(parts)
    return [int(v) for v in out.tolist()]


def exchange_exact(local, sizes, out, group=None):
    """Place every rank's `local` (sizes[r] elements) at its prefix offset of
    `out` (sum(sizes) elements, same dtype), moving exactly the shard bytes."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    base = [0]
    for s in sizes:
        base.append(base[-1] + s)
    assert local.numel() == sizes[rank] and out.numel() == base[-1], "shard sizes disagree"
    if world == 1:
        if out.data_ptr() != local.data_ptr():
            out.copy_(local)
        return out
    if len(set(sizes)) == 1 and out.is_cuda:
        if sizes[0]:
            dist.all_gather_into_tensor(out, local, group=group)
        return out
    if sizes[rank]:
        out[base[rank]:base[rank + 1]].copy_(local)
    ops = []
    for peer in range(world):
        if peer == rank:
            continue
        gpeer = dist.get_global_rank(group, peer) if group is not None else peer
        if sizes[rank]:
            ops.append(dist.P2POp(dist.isend, local, gpeer, group))
        if sizes[peer]:
            ops.append(dist.P2POp(dist.irecv, out[base[peer]:base[peer + 1]], gpeer, group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return out


def gather_stream(local_xdr, local_offsets=None, group=None, out=None, out_offsets=None):
    """Reassemble the rank-ordered concatenation of every rank's XDR shard.

    local_xdr: uint8 tensor (this rank's encoded records, exactly its bytes).
    local_offsets: optional int64 tensor [m+1] of record offsets inside the
    shard.  out / out_offsets: optional preallocated results (sizes must
    match).  Returns (stream, offsets) with offsets rebased to the full
    stream (or None)."""
    sizes = all_gather_ints(local_xdr.numel(), group)
    total = sum(sizes)
    if out is None:
        out = local_xdr.new_empty(total)
    stream = exchange_exact(local_xdr, sizes, out[:total], group)
    offs = None
    if local_offsets is not None:
        counts = all_gather_ints(local_offsets.numel() - 1, group)
        rank = dist.get_rank(group)
        n = sum(counts)
        if out_offsets is None:
            out_offsets = torch.empty(n + 1, dtype=torch.int64, device=local_offsets.device)
        mine = local_offsets[:-1].to(torch.int64) + sum(sizes[:rank])
        exchange_exact(mine, counts, out_offsets[:n], group)
        out_offsets[n] = total
        offs = out_offsets[:n + 1]
    return stream, offs


def encode_sharded(encode_shard, n, group=None):
    """Encode records [0, n) sharded over the group: encode_shard(lo, hi)
    returns (xdr uint8 tensor, offsets int64 tensor [hi-lo+1] or None) for
    this rank's range; the result is the full stream on every rank."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_range(n, world, rank)
    xdr, offs = encode_shard(lo, hi)
    return gather_stream(xdr, offs, group)


def decode_sharded(decode_shard, n, group=None):
    """Decode records [0, n) sharded over the group: decode_shard(lo, hi)
    decodes this rank's records (from the full stream and global record
    offsets it closes over) and returns (status, first_bad_global, err).
    Returns the reference's first error over all ranks: the minimum
    first_bad (ranks without an error report n)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_range(n, world, rank)
    status, first_bad, err = decode_shard(lo, hi)
    key = first_bad * 16 + err if status else n * 16
    best = min(all_gather_ints(key, group))
    if best >= n * 16:
        return 0, n, 0
    return best % 16, best // 16, best % 16


def stream_hash(t, chunk=1 << 24):
    """Position-weighted checksum of a byte tensor (sum of 32-bit words times
    their 1-based index, wrapping int64), chunked so the index vector stays
    small; equal streams give equal values on every rank."""
    n = t.numel()
    h = torch.zeros((), dtype=torch.int64, device=t.device)
    words = t[:n - n % 4].view(torch.int32)
    w = torch.arange(1, chunk + 1, dtype=torch.int64, device=t.device)
    for lo in range(0, words.numel(), chunk):
        c = words[lo:lo + chunk].to(torch.int64)
        h += (c * (w[:c.numel()] + lo)).sum()
    for i in range(n - n % 4, n):
        h += int(t[i]) * (i + 1)
    return int(h)
