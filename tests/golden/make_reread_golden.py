#!/usr/bin/env python3
"""Goldens for readGraphFromFile (OverlapGraph.cpp:1270-1367), the -s resume of
main.cpp:36-42: the REFERENCE itself (oracle/_ref/ref_harness reread, compiled
from /root/reference by oracle/Makefile) reads each fixture's committed
.unitig golden back, then sortEdges + saveGraphToFile.  Writes per fixture
  <name>.reread.gz         "#C nodes edges", every list in list order with its
                           reads, then the read location lists (as the unitig
                           dump of make_golden.py)
and records in <name>.json whether the re-saved file equals the input
("reread": {"file", "nodes", "edges", "resave_identical"}); when it differs the
re-saved file is kept as <name>.resaved.unitig.gz.  Build container only.
"""
import gzip
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import FIXTURES, fixture_input, load_meta  # noqa: E402


def main():
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    for name in FIXTURES:
        meta = load_meta(name)
        with tempfile.TemporaryDirectory() as td:
            uni = os.path.join(td, "in.unitig")
            with gzip.open(os.path.join(HERE, meta["unitig"]["file"]), "rb") as f, open(uni, "wb") as g:
                g.write(f.read())
            out = os.path.join(td, "out")
            subprocess.run([harness, "reread", fixture_input(name), str(meta["l"]), out, uni], check=True,
                           stdout=subprocess.DEVNULL)
            lists = open(out, "rb").read()
            resaved = open(out + ".unitig", "rb").read()
            same = resaved == open(uni, "rb").read()
        with gzip.GzipFile(os.path.join(HERE, f"{name}.reread.gz"), "wb", mtime=0) as f:
            f.write(lists)
        head = lists.split(b"\n", 1)[0].split()
        meta["reread"] = {"file": f"{name}.reread.gz", "nodes": int(head[1]), "edges": int(head[2]),
                          "resave_identical": same}
        if not same:
            with gzip.GzipFile(os.path.join(HERE, f"{name}.resaved.unitig.gz"), "wb", mtime=0) as f:
                f.write(resaved)
            meta["reread"]["resaved_file"] = f"{name}.resaved.unitig.gz"
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        print(name, meta["reread"])


if __name__ == "__main__":
    main()
