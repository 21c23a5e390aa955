import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
from metagenomics_amd import synth
from metagenomics_amd.overlap import Dataset, OverlapEngine, rows_to_tuples
from oracle import OracleDataset, sorted_tuples
# two reads: B = rc of a shifted window of A -> o=2 (A suffix == R_B prefix) and o=3 variants
X = synth.codes_to_strings(synth.random_genome(200, 3)[None, :], np.array([200]))[0]
cases = {"o2": [X[0:100], synth.revcomp_str(X[40:140])], "o0": [X[0:100], X[40:140]]}
eng = OverlapEngine(0)
for nm, seqs in cases.items():
    for k in (0, 12):
        ds = Dataset.from_strings(seqs, 30)
        eng.upload(ds); eng.build_index(30, k); eng.mark_contained()
        rows = rows_to_tuples(eng.rows(eng.find_overlaps()))
        od = OracleDataset.from_strings(seqs, 30); o, _, _, _ = od.overlaps(30)
        print(nm, "k", k, "gpu", rows.tolist(), "oracle", sorted_tuples(o).tolist())
        for i in (1, 2):
            s = ds.read(i); r = synth.revcomp_str(s)
            for o_, key in enumerate([s[:29], s[-29:], r[:29], r[-29:]]):
                print("   read", i, "o", o_, "lookup", eng.lookup(key), "oracle", od.lookup(30, key))
