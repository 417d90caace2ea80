#!/usr/bin/env python3
"""VGPR / spill / scratch of every non-counting instantiation of the persistent kernel in built trace objects
(register budget check after a traversal edit; WIDE 0 binary pairs, 1 quads by entry t, 2 quads in pair order; RAW 1 =
GPU-built scenes without cold records).  usage: scripts/kernel_resources.py real-time-gpu-ray-tracer_amd/build/trace_*.o"""
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
for obj in sys.argv[1:]:
    with tempfile.TemporaryDirectory() as d:
        fb = f"{d}/fb"
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", obj], check=True)
        co = f"{d}/co"
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fb}", f"--output={co}", "--unbundle"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    for e in notes.split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", e).group(1)
        m = re.search(r"render_persistent_kernelILb([01])ELi(\d)ELi(\d)ELi(\d)E", name)
        if not m or m.group(1) != "0":
            continue
        label = f"WPE {m.group(2)} WIDE {m.group(3)} RAW {m.group(4)}"
        g = lambda k: re.search(rf"\.{k}:\s+(\d+)", e).group(1)
        print(f"{obj.split('/')[-1]:22s} {label:22s} vgpr {g('vgpr_count'):>3} vspill {g('vgpr_spill_count'):>3} "
              f"sgpr {g('sgpr_count'):>3} sspill {g('sgpr_spill_count'):>3} scratch {g('private_segment_fixed_size')}")
