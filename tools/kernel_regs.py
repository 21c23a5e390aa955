"""Diagnostics: per-kernel VGPR/SGPR/spill/LDS of the gfx950 code objects
inside a built library (uncompressed clang offload bundles).
usage: kernel_regs.py [lib.so] [name-substring ...]"""
import re
import struct
import subprocess
import sys
import tempfile

lib = sys.argv[1] if len(sys.argv) > 1 else "metagenomics_amd/lib/libmgovl.so"
subs = sys.argv[2:]
d = open(lib, "rb").read()
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
pos = 0
while True:
    i = d.find(MAGIC, pos)
    if i < 0:
        break
    pos = i + len(MAGIC)
    n = struct.unpack_from("<Q", d, pos)[0]
    p = pos + 8
    for _ in range(n):
        off, size, tl = struct.unpack_from("<QQQ", d, p)
        triple = d[p + 24:p + 24 + tl].decode()
        p += 24 + tl
        if "gfx950" not in triple:
            continue
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(d[i + off:i + off + size])
            f.flush()
            t = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f.name],
                               capture_output=True, text=True).stdout
        for blk in t.split("  - .agpr_count")[1:]:
            g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
            name = g("name")
            dem = subprocess.run(["c++filt", name], capture_output=True,
                                 text=True).stdout.strip().replace("(anonymous namespace)::", "")
            if subs and not any(s in dem for s in subs):
                continue
            print(f"{dem[:70]:70s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>3} "
                  f"spill {g('vgpr_spill_count')} priv {g('private_segment_fixed_size')} "
                  f"lds {g('group_segment_fixed_size')}")
