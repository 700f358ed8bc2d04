#!/usr/bin/env python3
"""Identify the device code of libtmfwm.so's kernels, one id per kernel: sha256 (16 hex) over
the machine code of the kernel's own symbols in the TU's gfx950 code object (every template
instance of the family, e.g. embed_kernel<8, false> + embed_kernel<8, true>: the strip pass
and its list pass) and their kernel descriptors (register counts, LDS and scratch sizes; the
descriptor's code-entry offset, which only says where the linker placed the code, is masked).
The kernels make no PC-relative references (no s_getpc_b64 in the code objects), so a kernel's
bytes do not move with the code around it: an edit to embed_kernel<16> leaves the ids -- and
with them the counter profiles (profiles/valu.json) -- of extract_kernel<8> and <16> valid.
Written next to the library as libtmfwm.kernels.json by the Makefile; bench.py reports a
counter-derived figure only for the same code.
usage: kernel_ids.py <out.json> <tu.o>..."""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
BLOCKS = (4, 6, 8, 10, 12, 14, 16)
# mangled prefix of each family (tmf::embed_kernel<B, LIST>(EmbedArgs), tmf::extract_kernel<B, LIST>(ExtractArgs))
FAMILIES = {"embed_kernel": "_ZN3tmf12embed_kernelILi{b}EL", "extract_kernel": "_ZN3tmf14extract_kernelILi{b}EL"}
KD_ENTRY = slice(16, 24)  # kernel_code_entry_byte_offset in the 64-byte amdhsa kernel descriptor


def code_object(obj, d):
    fb = os.path.join(d, "fb.bin")
    co = os.path.join(d, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}", f"--targets={TARGET}",
                    f"--output={co}"], check=True)
    with open(co, "rb") as f:
        return co, f.read()


def sections(co):
    """name -> (address, file offset)"""
    out = subprocess.run([f"{LLVM}/llvm-readelf", "-S", "--wide", co], check=True, capture_output=True, text=True).stdout
    sec = {}
    for m in re.finditer(r"\]\s+(\S+)\s+\S+\s+([0-9a-f]+)\s+([0-9a-f]+)\s+([0-9a-f]+)", out):
        sec[m.group(1)] = (int(m.group(2), 16), int(m.group(3), 16))
    return sec


def symbols(co):
    """name -> (value, size, section index)"""
    out = subprocess.run([f"{LLVM}/llvm-readelf", "-s", "--wide", co], check=True, capture_output=True, text=True).stdout
    syms = {}
    for line in out.splitlines():
        p = line.split()
        if len(p) >= 8 and p[0].endswith(":") and p[3] in ("FUNC", "OBJECT"):
            syms[p[7]] = (int(p[1], 16), int(p[2]), p[6])
    return syms


def tu_kernels(obj):
    """family<B> -> id, for the kernels this TU defines"""
    with tempfile.TemporaryDirectory() as d:
        co, data = code_object(obj, d)
        sec, syms = sections(co), symbols(co)
    text, rodata = sec[".text"], sec[".rodata"]
    ids = {}
    for fam, pat in FAMILIES.items():
        for b in BLOCKS:
            pre = pat.format(b=b)
            names = sorted(n for n in syms if n.startswith(pre) and not n.endswith(".kd"))
            if not names:
                continue
            h = hashlib.sha256()
            for n in names:
                v, size, _ = syms[n]
                off = v - text[0] + text[1]
                h.update(n.encode() + data[off:off + size])
                kd = syms.get(n + ".kd")
                if kd:
                    ko = kd[0] - rodata[0] + rodata[1]
                    desc = bytearray(data[ko:ko + 64])
                    desc[KD_ENTRY] = bytes(8)
                    h.update(bytes(desc))
            ids[f"{fam}<{b}>"] = h.hexdigest()[:16]
    return ids


def main():
    if len(sys.argv) < 3 or sys.argv[1].startswith("-"):
        sys.exit("usage: kernel_ids.py OUT.json OBJ.o [OBJ.o ...]")
    out, objs = sys.argv[1], sys.argv[2:]
    kernels, tus = {}, {}
    for o in objs:
        k = tu_kernels(o)
        tus[os.path.splitext(os.path.basename(o))[0]] = sorted(k)
        for name, i in k.items():
            if name in kernels:
                raise SystemExit(f"kernel_ids: {name} defined in two TUs")
            kernels[name] = i
    with open(out, "w") as f:
        json.dump({"scheme": "per-kernel symbols + descriptors", "tu": tus, "kernels": kernels}, f, indent=1)


if __name__ == "__main__":
    main()
