"""Diagnostics: RCCL exchange mode with one rank; checks that every all-to-all
delivers exactly the bytes sent (world 1: recv == send) and that the row
count matches the fused path."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import torch.distributed as dist
from metagenomics_amd import synth
from metagenomics_amd.overlap import Dataset, OverlapEngine
from metagenomics_amd.sharded import TorchExchange, sharded_step

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
c, L = synth.uniform_read_set(n, 150, n * 150 // 20, seed=31)
ds = Dataset.from_codes(c, L, 50, nthreads=16)
torch.cuda.set_device(0)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29519")
dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1)

class Checked(TorchExchange):
    def all_to_all(self, sends, counts, rec_bytes):
        out = super().all_to_all(sends, counts, rec_bytes)
        nb = int(sum(int(x) for x in counts[0])) * rec_bytes
        same = torch.equal(sends[0][:nb], out[0][0][:nb])
        print(f"  a2a {nb/1e6:.1f} MB rec {rec_bytes}: equal={same}", flush=True)
        return out

fused = OverlapEngine(0); fused.upload(ds); fused.build_index(50, 31); fused.mark_contained(copy=False)
ref = fused.find_overlaps(); fused.close()
print("fused rows", ref, flush=True)
e = OverlapEngine(0); e.set_shard(0, 1, 0, 0); e.upload(ds)
for xc in (Checked(torch.device("cuda", 0)), TorchExchange(torch.device("cuda", 0))):
    for i in range(3):
        res = sharded_step([e], xc, 50, 31)
        print(type(xc).__name__, "step", i, "rows", res.rows[0][1], "diff", res.rows[0][1] - ref, flush=True)
dist.destroy_process_group()
