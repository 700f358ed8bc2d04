#!/usr/bin/env python3
"""Identify the device code of libtmfwm.so's kernels: sha256 (16 hex) of each TU's embedded
gfx950 code-object bundle (.hip_fatbin of the .o).  Written next to the library as
libtmfwm.kernels.json by the Makefile; profiles/valu.json records the id of the code its
counters measured, and bench.py reports a counter-derived figure only for the same code --
a rebuild that leaves a kernel's TU unchanged keeps its profile valid.
usage: kernel_ids.py <out.json> <tu.o>..."""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

OBJCOPY = "/opt/rocm/lib/llvm/bin/llvm-objcopy"
# which TU holds which kernel (tmfwm_embed8.hip: embed_kernel<8> alone; the rest in tmfwm_kernels.hip)
TU_OF = {"embed_kernel<8>": "tmfwm_embed8"}
BLOCKS = (4, 6, 8, 10, 12, 14, 16)


def fatbin_id(obj):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "fb.bin")
        subprocess.run([OBJCOPY, f"--dump-section=.hip_fatbin={out}", obj], check=True)
        with open(out, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]


def main():
    out, objs = sys.argv[1], sys.argv[2:]
    tus = {os.path.splitext(os.path.basename(o))[0]: fatbin_id(o) for o in objs}
    kernels = {}
    for b in BLOCKS:
        for k in (f"embed_kernel<{b}>", f"extract_kernel<{b}>"):
            tu = TU_OF.get(k, "tmfwm_kernels")
            if tu in tus:
                kernels[k] = tus[tu]
    with open(out, "w") as f:
        json.dump({"tu": tus, "kernels": kernels}, f, indent=1)


if __name__ == "__main__":
    main()
