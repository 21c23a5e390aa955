import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from metagenomics_amd import overlap, synth
overlap.LIB_PATH = os.path.join(ROOT, "tools", sys.argv[1] if len(sys.argv) > 1 else "dbg_lib", "libmgovl.so")
from metagenomics_amd.overlap import Dataset, OverlapEngine, rows_to_tuples
X = synth.codes_to_strings(synth.random_genome(200, 3)[None, :], np.array([200]))[0]
seqs = [X[0:100], X[40:140]]
eng = OverlapEngine(0)
ds = Dataset.from_strings(seqs, 30)
eng.upload(ds); eng.build_index(30, 0); eng.mark_contained()
print(rows_to_tuples(eng.rows(eng.find_overlaps())).tolist(), flush=True)
seqs = [X[0:100], synth.revcomp_str(X[30:80])]   # rc containment, mixed lengths
ds = Dataset.from_strings(seqs, 30)
eng.upload(ds); eng.build_index(30, 0); print("super", eng.mark_contained().tolist(), flush=True)
