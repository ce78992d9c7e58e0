"""Multi-GPU plumbing: utterance sharding and the result gather.

Utterances are independent, so rank r of N processes owns a contiguous shard and runs
the whole encode/decode path with no data-path collective. The only exchange is the
result gather: per-utterance packet bytes (and a few f32 stats) to rank 0, done with
``all_gather`` of lengths then of zero-padded byte tensors — RCCL over xGMI when the
process group is ``nccl`` (tensors on the rank's GPU), gloo on CPU in tests. A few KB
per rank: latency-bound, never on the timed path's critical loop.
"""
import torch
import torch.distributed as dist


def shard(rank: int, world: int, total: int):
    """[begin, end) of rank's utterances; shards differ in size by at most one."""
    base, extra = divmod(total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def gather_packets(packets, device, group=None):
    """All-gather a list of packet byte strings (None = no packet) from every rank;
    returns the flattened list in rank order on every rank."""
    world = dist.get_world_size(group)
    blobs = [b"" if p is None else p for p in packets]
    lens = torch.tensor([len(b) for b in blobs] + [-1 if p is None else 0 for p in packets],
                        dtype=torch.int64, device=device)
    n_local = torch.tensor([len(blobs)], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(counts, n_local, group=group)
    counts = [int(c.item()) for c in counts]
    maxn = max(counts)
    pad_lens = torch.zeros(2 * maxn, dtype=torch.int64, device=device)
    pad_lens[:len(blobs)] = lens[:len(blobs)]
    pad_lens[maxn:maxn + len(blobs)] = lens[len(blobs):]
    all_lens = [torch.zeros_like(pad_lens) for _ in range(world)]
    dist.all_gather(all_lens, pad_lens, group=group)
    total_bytes = [int(l[:maxn].sum().item()) for l in all_lens]
    maxb = max(max(total_bytes), 1)
    payload = torch.zeros(maxb, dtype=torch.uint8, device=device)
    flat = b"".join(blobs)
    if flat:
        payload[:len(flat)] = torch.frombuffer(bytearray(flat), dtype=torch.uint8).to(device)
    all_payload = [torch.zeros_like(payload) for _ in range(world)]
    dist.all_gather(all_payload, payload, group=group)
    out = []
    for r in range(world):
        data = bytes(all_payload[r].cpu().numpy().tobytes())
        ls = all_lens[r].cpu().tolist()
        pos = 0
        for i in range(counts[r]):
            n, none = ls[i], ls[maxn + i]
            out.append(None if none == -1 else data[pos:pos + n])
            pos += n
    return out


def gather_stats(stats: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather per-utterance f32 statistics [n_local][k] (rms, mean f0, voiced hops)
    from every rank -> [total][k] in rank order, on every rank (ranks may hold different
    n_local). The tensor stays on its device: RCCL for a GPU tensor under ``nccl``."""
    world = dist.get_world_size(group)
    stats = stats.to(torch.float32).contiguous()
    n_local = torch.tensor([stats.shape[0]], dtype=torch.int64, device=stats.device)
    counts = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(counts, n_local, group=group)
    counts = [int(c.item()) for c in counts]
    maxn = max(max(counts), 1)
    pad = torch.zeros(maxn, stats.shape[1], dtype=torch.float32, device=stats.device)
    pad[:stats.shape[0]] = stats
    parts = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, counts)])


def gather_values(values, device, group=None):
    """All-gather a variable-length list of floats from every rank (config 5's per-block
    and per-phrase latencies) -> one flat list in rank order, on every rank."""
    t = torch.tensor([float(v) for v in values], dtype=torch.float64).reshape(-1, 1)
    g = gather_stats(t.to(device), group)   # float32 keeps µs at these magnitudes
    return [float(v) for v in g.reshape(-1).cpu().tolist()]


def gather_results(packets, stats: torch.Tensor, device, group=None):
    """The result gather of SURVEY §8(e): packet bytes and per-utterance stats."""
    return gather_packets(packets, device, group), gather_stats(stats, group)
