"""Image-level sharding of a batch over the GPUs of a node (BASELINE
configs[3]: 64 frames over 8 MI355X) and the final gather of the encoded
JPEG byte strings -- the only collective on the path (RCCL over xGMI when
the process group is "nccl"; gloo on CPU in the tests).

Frames are independent units: rank r encodes frames r, r + world, ...; no
data moves between GPUs until the byte strings are gathered.
"""


def shard(n_frames, world, rank):
    """Indices of the frames rank `rank` encodes (round-robin)."""
    return list(range(rank, n_frames, world))


def gather_bytes(blobs, dist, device):
    """All-gathers each rank's list of byte strings; returns the list of
    every rank's list (rank order).  Two collectives: sizes, then a padded
    byte buffer.  `device` is where the buffers live ("cuda:N" for RCCL,
    "cpu" for gloo)."""
    import torch

    world = dist.get_world_size()
    lens = torch.tensor([len(b) for b in blobs], dtype=torch.int64, device=device)
    count = torch.tensor([len(blobs)], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(count) for _ in range(world)]
    dist.all_gather(counts, count)
    max_count = int(max(int(c.item()) for c in counts))
    lens_p = torch.zeros(max_count, dtype=torch.int64, device=device)
    lens_p[:len(blobs)] = lens
    all_lens = [torch.zeros_like(lens_p) for _ in range(world)]
    dist.all_gather(all_lens, lens_p)
    total = [int(l.sum().item()) for l in all_lens]
    buf = torch.zeros(max(max(total), 1), dtype=torch.uint8, device=device)
    blob = b"".join(blobs)
    if blob:
        buf[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(device)
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    out = []
    for r in range(world):
        n = int(counts[r].item())
        data = bytes(bufs[r][:total[r]].cpu().numpy().tobytes())
        items, off = [], 0
        for l in all_lens[r][:n].tolist():
            items.append(data[off:off + l])
            off += l
        out.append(items)
    return out
