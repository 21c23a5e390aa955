"""Diagnostics: torch.distributed all_to_all_single (RCCL, world 1) integrity
for large byte buffers, by element type and size."""
import os, time, torch, torch.distributed as dist
torch.cuda.set_device(0)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29521")
dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1)
for mb in (256, 1000, 1100, 1600, 2100, 2800):
    nb = mb * 1_000_000 // 16 * 16
    src = torch.randint(0, 255, (nb,), dtype=torch.uint8, device="cuda")
    for dt in (torch.uint8, torch.int32, torch.int64):
        s = src.view(dt)
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, output_split_sizes=[s.numel()], input_split_sizes=[s.numel()])
        torch.cuda.synchronize()
        ok1 = torch.equal(r, s)
        time.sleep(0.5); torch.cuda.synchronize()
        ok2 = torch.equal(r, s)
        r2 = torch.empty_like(s)
        dist.all_to_all_single(r2, s)
        torch.cuda.synchronize()
        print(f"{mb} MB {dt}: split-form equal={ok1} after-sleep={ok2}; even-form equal={torch.equal(r2, s)}", flush=True)
        del r, r2
    del src
dist.destroy_process_group()
