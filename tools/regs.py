#!/usr/bin/env python3
"""Register / scratch / occupancy table of the gfx950 kernels (from the compiler's
kernel-resource-usage remarks): python tools/regs.py [extra hipcc flags] [-k filter]."""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
CSRC = ROOT + "/thatsmyface_amd/csrc"


def main():
    args = sys.argv[1:]
    filt = None
    if "-k" in args:
        i = args.index("-k")
        filt = args[i + 1]
        del args[i:i + 2]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
           "-fno-slp-vectorize", "--cuda-device-only", "-c", "tmfwm_kernels.hip", "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"] + args
    out = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True).stderr
    cmd8 = [c if c != "tmfwm_kernels.hip" else "tmfwm_embed8.hip" for c in cmd] + ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
    out += subprocess.run(cmd8, cwd=CSRC, capture_output=True, text=True).stderr
    for tu in ("tmfwm_rank1.hip", "tmfwm_rank1_lists.hip"):
        out += subprocess.run([c if c != "tmfwm_kernels.hip" else tu for c in cmd], cwd=CSRC, capture_output=True,
                              text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill|LDS Size \[bytes/block\]): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k.split(" ")[0] + ("_spill" if "Spill" in k else "")] = v
    for r in rows:
        n = r["name"]
        if filt and not re.search(filt, n):
            continue
        n = re.sub(r"^_ZN3tmf\d+", "", n)
        print(f"{n[:48]:48s} vgpr {r.get('VGPRs','?'):>4s} spill {r.get('VGPRs_spill','?'):>3s} "
              f"scratch {r.get('ScratchSize','?'):>4s} occ {r.get('Occupancy','?'):>2s} lds {r.get('LDS','?')}")


if __name__ == "__main__":
    main()
