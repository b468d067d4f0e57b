"""Multi-GPU layout of the batched STFT (BASELINE config 5).

Channels are independent, so the path shards without any data-path exchange:
rank r owns a contiguous channel range and runs the single-GPU kernels on it
(one process per GPU, torch.distributed for rendezvous only).  The only
collective is the optional gather of the spectrogram rows to one rank that
config 5 asks for ("RCCL gather over xGMI"): on the nccl backend (= RCCL on
ROCm) `dist.gather` is point-to-point over xGMI; on gloo it is the same call
on CPU tensors, which is how the CPU test suite exercises this module.
"""
import torch
import torch.distributed as dist


def channel_shard(total, world, rank):
    """Contiguous channel range [lo, hi) of `rank`; rank order == channel order,
    sizes differ by at most one."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    base, rem = divmod(int(total), int(world))
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_sizes(total, world):
    return [b - a for a, b in (channel_shard(total, world, r) for r in range(world))]


def frame_shard(frames, world, rank):
    """Contiguous frame range [lo, hi) of `rank` for one long signal (SURVEY 8e,
    config 3 sharded): whole frame pairs per rank, so every lo is even and each
    rank's rows are bit-identical to the unsharded spectrogram (the kernels
    transform frames (2j, 2j+1) together)."""
    plo, phi = channel_shard((int(frames) + 1) // 2, world, rank)
    return min(2 * plo, frames), min(2 * phi, frames)


def frame_shard_sizes(frames, world):
    return [b - a for a, b in (frame_shard(frames, world, r) for r in range(world))]


GATHER_SLAB_BYTES = 1 << 30


def gather_rows(local, total, dst=0, group=None, out=None, sizes=None):
    """Gather every rank's [ch_r, ...] block into one [total, ...] tensor on
    rank `dst` (None elsewhere).  Equal shards land directly in `out` (or a
    new tensor) with no extra copy; uneven shards are padded to the largest
    one for the collective and trimmed on the destination.  `sizes`: the
    per-rank leading sizes (default: the channel_shard layout)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = shard_sizes(total, world) if sizes is None else list(sizes)
    if len(sizes) != world or sum(sizes) != total:
        raise ValueError(f"shard sizes {sizes} do not cover {total} rows on {world} ranks")
    if local.shape[0] != sizes[rank]:
        raise ValueError(f"rank {rank} holds {local.shape[0]} channels, layout says {sizes[rank]}")
    cmax = max(sizes)
    if min(sizes) == cmax and cmax > 0:
        # slabs of whole channels, at most ~1 GiB per rank per collective: keeps
        # every message far below 2^31 elements (a config-5 shard is 14.7 GB)
        row_bytes = max(1, local[0].numel() * local.element_size())
        step = max(1, min(cmax, GATHER_SLAB_BYTES // row_bytes))
        loc = local.contiguous()
        if rank == dst:
            if out is None:
                out = torch.empty((total,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
            ov = out.view((world, cmax) + tuple(local.shape[1:]))
        for i0 in range(0, cmax, step):
            i1 = min(cmax, i0 + step)
            if rank == dst:
                dist.gather(loc[i0:i1], gather_list=[ov[r, i0:i1] for r in range(world)], dst=dst, group=group)
            else:
                dist.gather(loc[i0:i1], dst=dst, group=group)
        return out if rank == dst else None
    if local.shape[0] < cmax:
        pad = torch.zeros((cmax - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        send = torch.cat([local, pad], 0)
    else:
        send = local.contiguous()
    if rank == dst:
        bufs = [torch.empty_like(send) for _ in range(world)]
        dist.gather(send, gather_list=bufs, dst=dst, group=group)
        return torch.cat([b[:s] for b, s in zip(bufs, sizes)], 0)
    dist.gather(send, dst=dst, group=group)
    return None


def gather_rows_stream(local, total, sink, dst=0, group=None, sizes=None, slab_bytes=GATHER_SLAB_BYTES):
    """gather_rows without the [total, ...] destination: rank `dst` receives
    slabs of at most ~slab_bytes per rank into one reusable staging buffer and
    hands each rank's piece to sink(first_row, block) in row order (e.g.
    host_sink: straight into a pinned host tensor, so config 5's 118 GB never
    has to fit on one GPU next to its own shard).  Ranks with fewer rows pad
    their slabs; only real rows reach the sink."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = shard_sizes(total, world) if sizes is None else list(sizes)
    if len(sizes) != world or sum(sizes) != total:
        raise ValueError(f"shard sizes {sizes} do not cover {total} rows on {world} ranks")
    if local.shape[0] != sizes[rank]:
        raise ValueError(f"rank {rank} holds {local.shape[0]} channels, layout says {sizes[rank]}")
    cmax = max(sizes)
    if cmax == 0:
        return
    firsts = [sum(sizes[:r]) for r in range(world)]
    tail = tuple(local.shape[1:])
    row_bytes = max(1, int(torch.Size(tail).numel()) * local.element_size())
    step = max(1, min(cmax, int(slab_bytes) // row_bytes))
    loc = local.contiguous()
    send = torch.empty((step,) + tail, dtype=local.dtype, device=local.device)
    stage = torch.empty((world, step) + tail, dtype=local.dtype, device=local.device) if rank == dst else None
    for i0 in range(0, cmax, step):
        i1 = min(cmax, i0 + step)
        mine = max(0, min(i1, sizes[rank]) - i0)   # real rows of this slab on this rank
        if mine:
            send[:mine].copy_(loc[i0:i0 + mine])
        if mine < i1 - i0:
            send[mine:i1 - i0].zero_()
        if rank == dst:
            dist.gather(send[:i1 - i0], gather_list=[stage[r, :i1 - i0] for r in range(world)], dst=dst, group=group)
            for r in range(world):
                real = max(0, min(i1, sizes[r]) - i0)
                if real:
                    sink(firsts[r] + i0, stage[r, :real])
        else:
            dist.gather(send[:i1 - i0], dst=dst, group=group)


def host_sink(out):
    """A gather_rows_stream sink that copies each block into the host tensor
    `out` ([total, ...], ideally pinned) at its row position."""
    def sink(first, block):
        out[first:first + block.shape[0]].copy_(block)
    return sink


def gather_rows_half(local, total, nfft, dst=0, group=None, out=None, pack=None, unpack=None):
    """gather_rows for magnitude rows [ch, frames, nfft] of real frames, sending
    bins 0..nfft/2 only (SURVEY 8e row note 1: half the xGMI bytes of config 5's
    gather).  The library's power rows are already nfft/2+1 wide: gather those
    with gather_rows directly.  Each rank packs its rows, the packed rows are gathered,
    and rank `dst` expands them by mirror symmetry.  pack / unpack default to
    the library's device kernels (vv_dsp_spectrogram_{pack,unpack}_half_device);
    for fused-kernel rows the result equals gather_rows bit for bit."""
    if pack is None or unpack is None:
        import vvdsp_amd as vv
        pack = pack or (lambda t: vv.pack_half(t, nfft))
        unpack = unpack or (lambda t, o: vv.unpack_half(t, nfft, out=o))
    half = pack(local)
    got = gather_rows(half, total, dst=dst, group=group)
    del half
    if got is None:
        return None
    if out is None:
        out = torch.empty(tuple(got.shape[:-1]) + (nfft,), dtype=got.dtype, device=got.device)
    unpack(got, out)
    return out


def gather_frames(local, frames, dst=0, group=None):
    """Gather a single signal's frame shards ([f_r, width] per rank, frame_shard
    layout) into the whole [frames, width] spectrogram on rank `dst`."""
    world = dist.get_world_size(group)
    return gather_rows(local, frames, dst=dst, group=group, sizes=frame_shard_sizes(frames, world))
