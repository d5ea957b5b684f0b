"""ISA fingerprint of the step kernels: per kernel symbol, the VGPR / SGPR / scratch counts and the
instruction-mnemonic histogram of the gfx950 code object, so a source refactor can be shown to leave the
shipped kernels' machine code unchanged.

    python tools/isa_fingerprint.py [src.hip] > fp.json
    python tools/isa_fingerprint.py --diff a.json b.json
"""
from __future__ import annotations

import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gameoflifewithactors_amd", "csrc")


def fingerprint(src: str, defines=()) -> dict:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-x", "hip",
               "--cuda-device-only", "-S", "-I", os.path.join(ROOT, "include"), "-I", CSRC, src, "-o", out]
        cmd += [f"-D{x}" for x in defines]
        subprocess.run(cmd, check=True)
        text = open(out).read()
    kernels = {}
    cur = None
    for line in text.splitlines():
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m and "gol_stream_step" in line:
            cur = m.group(1)
            kernels[cur] = {"hist": collections.Counter()}
            continue
        if cur is None:
            continue
        s = line.strip()
        if s.startswith(".Lfunc_end"):
            cur = None
            continue
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        kernels[cur]["hist"][s.split()[0]] += 1
    # resource usage from the metadata
    for name, k in kernels.items():
        m = re.search(re.escape(name) + r"\.num_vgpr, (\d+)", text)
        k["vgpr"] = int(m.group(1)) if m else None
        m = re.search(re.escape(name) + r"\.private_seg_size, (\d+)", text)
        k["scratch"] = int(m.group(1)) if m else None
        k["n_instr"] = sum(k["hist"].values())
        k["hist"] = dict(sorted(k["hist"].items()))
    return kernels


def main():
    if len(sys.argv) == 4 and sys.argv[1] == "--diff":
        a, b = (json.load(open(p)) for p in sys.argv[2:])
        same = 0
        for k in sorted(set(a) | set(b)):
            if k not in a or k not in b:
                print(("only in a: " if k in a else "only in b: ") + k)
            elif a[k] != b[k]:
                print(f"DIFF {k}: vgpr {a[k]['vgpr']} -> {b[k]['vgpr']}, instr {a[k]['n_instr']} -> {b[k]['n_instr']}")
            else:
                same += 1
        print(f"{same} kernels identical")
        return
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(CSRC, "gol_step.hip")
    json.dump(fingerprint(src), sys.stdout, indent=1)


if __name__ == "__main__":
    main()
