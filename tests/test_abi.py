"""The C-ABI library loads and exports every symbol include/*.h declares; no
compute is attempted without a GPU."""
import ctypes
import glob
import os
import re

import pytest

from conftest import ROOT, gpu_available
from metagenomics_amd import overlap


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b((?:mg|mgh)_\w+)\s*\(", txt, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def test_headers_declare_the_boundary():
    names = declared_functions()
    for must in ["mg_create", "mg_upload_reads_packed", "mg_build_index", "mg_mark_contained",
                 "mg_find_overlaps", "mg_copy_rows", "mg_lookup_key", "mg_set_shard", "mgh_dataset_from_files"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(overlap.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_edge_struct_is_12_bytes():
    assert overlap.EDGE_DTYPE.itemsize == 12


@pytest.mark.skipif(gpu_available(), reason="only meaningful without a GPU")
def test_no_gpu_fails_loudly():
    assert overlap.device_count() == 0
    with pytest.raises(overlap.MgError):
        overlap.OverlapEngine(0)
