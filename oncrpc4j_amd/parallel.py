"""parallel.py — record-sharded XDR encode/decode across GPUs (one process per GPU).

Records are independent (no cross-record state in org.dcache.oncrpc4j.xdr.Xdr;
an XdrAble encodes into the stream in order), so a batch of N
records shards into contiguous record ranges, rank r owning
[r*N/G, (r+1)*N/G).  Encode and decode need no collective.  Reassembling
one contiguous XDR stream (BASELINE configs[4]) is the only exchange:

* fixed-size records: every shard has the same byte count -> one rank-ordered
  all-gather (RCCL `all_gather_into_tensor` over xGMI) is exactly the
  single-GPU stream;
* variable-size records: all-gather of the per-rank byte counts, then an
  all-gather of shards padded to the largest, compacted in rank order (RCCL
  has no all-gather-v).  Record offsets are rebased by the exclusive prefix of
  the shard sizes.

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


def _all_gather_sizes(x, group=None, dev=None):
    world = dist.get_world_size(group)
    dev = dev or _coll_device(group)
    mine = torch.tensor([x], dtype=torch.int64, device=dev)
    out = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(out, mine, group=group)
    return [int(t.item()) for t in out]


def _all_gather_padded(local, size, group=None):
    world = dist.get_world_size(group)
    if local.numel() < size:
        pad = torch.zeros(size - local.numel(), dtype=local.dtype, device=local.device)
        local = torch.cat([local, pad])
    parts = [torch.empty(size, dtype=local.dtype, device=local.device) for _ in range(world)]
    if local.is_cuda and hasattr(dist, "all_gather_into_tensor"):
        flat = torch.empty(world * size, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(flat, local, group=group)
        return list(flat.view(world, size))
    dist.all_gather(parts, local, group=group)
    return parts


def gather_stream(local_xdr, local_offsets=None, group=None):
    """Reassemble the rank-ordered concatenation of every rank's XDR shard.

    local_xdr: uint8 tensor (this rank's encoded records, exactly its bytes).
    local_offsets: optional int64 tensor [m+1] of record offsets inside the
    shard.  Returns (stream, offsets) with offsets rebased to the full stream
    (or None)."""
    sizes = _all_gather_sizes(local_xdr.numel(), group)
    big = max(sizes)
    if big == 0:
        stream = local_xdr.new_empty(0)
    elif all(s == big for s in sizes):
        stream = torch.cat(_all_gather_padded(local_xdr, big, group)) if len(sizes) > 1 else local_xdr
    else:
        parts = _all_gather_padded(local_xdr, big, group)
        stream = torch.cat([p[:s] for p, s in zip(parts, sizes)])
    offs = None
    if local_offsets is not None:
        counts = _all_gather_sizes(local_offsets.numel() - 1, group)
        rank = dist.get_rank(group)
        base = sum(sizes[:rank])
        mine = (local_offsets[:-1] + base).to(torch.int64)
        gathered = _all_gather_padded(mine, max(max(counts), 1), group)
        pieces = [g[:c] for g, c in zip(gathered, counts)]
        end = torch.tensor([sum(sizes)], dtype=torch.int64, device=local_offsets.device)
        offs = torch.cat(pieces + [end])
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
    key = first_bad * 16 + (err if status else 0) if status else n * 16
    keys = _all_gather_sizes(key, group)
    best = min(keys)
    if best >= n * 16:
        return 0, n, 0
    return best % 16, best // 16, best % 16
