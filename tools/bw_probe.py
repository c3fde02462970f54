#!/usr/bin/env python3
"""Practical HBM copy bandwidth on this GPU at the working-set sizes of the
Compare pass (torch device-to-device copy, HIP-event timed)."""
import torch


def main():
    for mb in (8, 25, 50, 100, 400, 1600):
        n = mb * (1 << 20) // 4
        a = torch.empty(n, dtype=torch.float32, device="cuda").uniform_()
        b = torch.empty_like(a)
        for _ in range(3):
            b.copy_(a)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 50
        e0.record()
        for _ in range(reps):
            b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"copy {mb:5d} MB: {ms * 1e3:8.1f} us  {2 * mb * (1 << 20) / ms / 1e6:8.1f} GB/s (read+write)")


if __name__ == "__main__":
    main()
