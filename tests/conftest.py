import gzip
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

FIXTURES = ["small", "mixed", "highdup", "tandem", "tworead", "dirty", "wrapped", "branchy", "longreads"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def _ensure_built():
    lib = os.path.join(ROOT, "metagenomics_amd", "lib", "libmgovl.so")
    orc = os.path.join(ROOT, "oracle", "build", "libmgoracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "metagenomics_amd", "csrc"), "-j8"], check=True)
    if not os.path.exists(orc):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"], check=True)


_ensure_built()


def load_meta(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


def fixture_input(name, tmp_path_factory=None):
    """Decompress the fixture's input into a temp file; returns its path."""
    meta = load_meta(name)
    src = os.path.join(GOLDEN, meta["input"])
    d = os.environ.get("MG_TEST_TMP") or "/tmp/mg_golden"
    os.makedirs(d, exist_ok=True)
    dst = os.path.join(d, meta["input"][:-3])
    if not os.path.exists(dst):
        part = "%s.%d.part" % (dst, os.getpid())  # parallel workers (pytest -n) each write their own
        with gzip.open(src, "rb") as f, open(part, "wb") as g:
            g.write(f.read())
        os.replace(part, dst)
    return dst


def golden_rows(name) -> np.ndarray:
    meta = load_meta(name)
    with gzip.open(os.path.join(GOLDEN, meta["edges_file"]), "rt") as f:
        txt = f.read().split()
    arr = np.array(txt, dtype=np.int64).reshape(-1, 4) if txt else np.zeros((0, 4), np.int64)
    return arr


def rows_sha256(tuples: np.ndarray) -> str:
    import hashlib

    h = hashlib.sha256()
    h.update("".join("%d %d %d %d\n" % tuple(r) for r in tuples.tolist()).encode())
    return h.hexdigest()


def ids_sha256(read_fn, n) -> str:
    import hashlib

    h = hashlib.sha256()
    for i in range(1, n + 1):
        h.update(("%d %s\n" % (i, read_fn(i))).encode())
    return h.hexdigest()


def gpu_available() -> bool:
    try:
        from metagenomics_amd import overlap

        return overlap.device_count() > 0
    except Exception:
        return False
