#!/usr/bin/env python3
"""Static check of every LDS-DMA load (global_load_lds_*) in the device assembly.

global_load_lds takes its LDS destination base from M0.  For each one this walks back
through its basic block to the instruction that last wrote M0 and reports:
  - no M0 write in the block (the base comes from another block: flagged);
  - anything between that write and the load that also writes M0, or that is a
    scratch (spill) access -- the two ways round 2's spilling 4-waves/SIMD variant
    of k_env_step_bits128 could have disturbed the DMA;
  - the M0 values used per kernel (the LDS byte offsets the DMA writes);
  - a kernel that issues LDS-DMA loads and uses scratch (spills): the condition the
    faulting variant had and the shipped kernels must not have.

Usage: isa_lds_dma_check.py [file.s ...]   (default: compile the shipped sources to
assembly under build/asm, as `make -C safelife-k2_amd/csrc asm` does, and check
them).  Exit status 1 when any load is flagged.
"""
import glob
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "safelife-k2_amd", "csrc")


def compile_asm(out_dir):
    os.makedirs(out_dir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "sl_bits*.hip")))     # the LDS-DMA kernels
    for s in srcs:
        out = os.path.join(out_dir, os.path.basename(s)[:-4] + ".s")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3",
                               "-std=c++17", "-fPIC", "-munsafe-fp-atomics", "-fno-gpu-rdc",
                               "-ffp-contract=off", "--cuda-device-only", "-S", s, "-o", out],
                              stderr=subprocess.DEVNULL)
    return sorted(glob.glob(os.path.join(out_dir, "*.s")))


M0_WRITE = re.compile(r"^\s*s_\w+\s+m0\b")
LABEL = re.compile(r"^(\.LBB\w+|_Z\w+):")
BRANCH = re.compile(r"^\s*s_(branch|cbranch_\w+|setpc|swappc|endpgm)\b")


def check(path):
    issues, loads = [], 0
    fn, block = None, []
    m0_values, dma_fns = {}, set()
    for raw in open(path):
        m = re.match(r"\s*\.amdhsa_private_segment_fixed_size (\d+)", raw)
        if m and fn in dma_fns and int(m.group(1)) > 0:
            issues.append((fn, "uses %s B of scratch per lane (spills) beside LDS-DMA loads"
                           % m.group(1), ""))
        line = raw.split(";")[0].rstrip()
        lab = LABEL.match(raw)
        if lab:
            if lab.group(1).startswith("_Z"):
                fn = lab.group(1)
            block = []
            continue
        if not line.strip():
            continue
        if "global_load_lds" in line or "buffer_load" in line and " lds" in line:
            loads += 1
            dma_fns.add(fn)
            j = len(block) - 1
            between = []
            while j >= 0 and not M0_WRITE.match(block[j]):
                between.append(block[j].strip())
                j -= 1
            if j < 0:
                issues.append((fn, "M0 not written in the load's block", line.strip()))
            else:
                m0_values.setdefault(fn, set()).add(block[j].split()[-1])
                bad = [b for b in between if M0_WRITE.match(b) or "m0" in b.split()
                       or b.startswith(("scratch_", "buffer_store", "buffer_load"))
                       and "off offset" in b]
                if bad:
                    issues.append((fn, "between the M0 write and the load: %s" % bad,
                                   line.strip()))
        block.append(line)
        if BRANCH.match(line):
            block = []
    return loads, issues, m0_values


def main(paths):
    if not paths:
        paths = compile_asm(os.path.join(REPO, "build", "asm"))
    total, bad = 0, []
    for p in paths:
        n, issues, m0 = check(p)
        total += n
        bad += [(os.path.basename(p),) + i for i in issues]
        for fn, vals in sorted(m0.items()):
            print("%s %s: M0 = %s" % (os.path.basename(p), fn[:60], ", ".join(sorted(vals))))
    for b in bad:
        print("FLAG", *b)
    print("%d LDS-DMA loads checked, %d flagged" % (total, len(bad)))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
