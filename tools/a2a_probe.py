"""Diagnostics: torch.distributed all_to_all_single (RCCL, world 1) integrity
for large buffers, by element type and size.  For each case:
equal or not, and for a corrupted result the first differing byte offset and
the differing fraction, so a 2^30-byte internal boundary shows up as such.
Also: the same payload as four equal-split calls of <= 512 MiB (what
metagenomics_amd/sharded.py does), all_gather_into_tensor and broadcast of
the same size, and a plain device copy."""
import os
import time

import torch
import torch.distributed as dist

torch.cuda.set_device(0)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29521")
dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1)


def diff(r, s):
    a, b = r.view(torch.uint8), s.view(torch.uint8)
    ne = a != b
    n = int(ne.sum())
    if n == 0:
        return "equal"
    first = int(torch.nonzero(ne)[0])
    return f"DIFF first_byte={first} (2^30={1 << 30}) frac={n / a.numel():.4f}"


for mb in (900, 1000, 1073, 1074, 1100, 1600, 2100):
    nb = mb * 1_000_000 // 64 * 64
    src = torch.randint(0, 255, (nb,), dtype=torch.uint8, device="cuda")
    for dt in (torch.uint8, torch.int64):
        s = src.view(dt)
        r = torch.empty_like(s)
        t0 = time.perf_counter()
        dist.all_to_all_single(r, s)
        torch.cuda.synchronize()
        dt_ms = (time.perf_counter() - t0) * 1e3
        print(f"{mb} MB {dt} bytes={nb} (<2^31: {nb < 2**31}) elems={s.numel()}: a2a {diff(r, s)} "
              f"({dt_ms:.1f} ms)", flush=True)
        del r
    # the same payload in four equal-split rounds (the exchange mode's chunking)
    s = src.view(torch.int64)
    r = torch.empty_like(s)
    q = s.numel() // 4
    for i in range(4):
        hi = s.numel() if i == 3 else (i + 1) * q
        dist.all_to_all_single(r[i * q: hi], s[i * q: hi])
    torch.cuda.synchronize()
    print(f"{mb} MB int64 in 4 rounds: {diff(r, s)}", flush=True)
    g = torch.empty_like(s)
    dist.all_gather_into_tensor(g, s)
    torch.cuda.synchronize()
    print(f"{mb} MB int64 all_gather_into_tensor: {diff(g, s)}", flush=True)
    b = s.clone()
    dist.broadcast(b, 0)
    torch.cuda.synchronize()
    print(f"{mb} MB int64 broadcast: {diff(b, s)}", flush=True)
    c = torch.empty_like(s)
    c.copy_(s)
    torch.cuda.synchronize()
    print(f"{mb} MB int64 device copy: {diff(c, s)}", flush=True)
    del src, s, r, g, b, c
dist.destroy_process_group()
