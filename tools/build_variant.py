#!/usr/bin/env python3
"""Build an A/B variant of libsafelife_hip.so from patched sources (timing experiments).

Usage: build_variant.py <spec.py> [name ...]
spec.py defines VARIANTS = {name: [(file, old, new), ...]}.  For each variant: copies safelife-k2_amd/csrc and include/ to /tmp/slvar/<name>, applies the literal
replacements (each must match), builds with the shipped Makefile's flags into
variants/<name>.so (git-ignored, travels to the GPU box; load it with
SAFELIFE_HIP_LIB=variants/<name>.so).  Prints the step kernels' register use.
"""
import os
import re
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(name, reps):
    root = os.path.join("/tmp/slvar", name)
    shutil.rmtree(root, ignore_errors=True)
    shutil.copytree(os.path.join(REPO, "safelife-k2_amd", "csrc"), os.path.join(root, "pkg", "csrc"))
    shutil.copytree(os.path.join(REPO, "include"), os.path.join(root, "include"))
    for f, old, new in reps:
        p = os.path.join(root, "pkg", "csrc", f)
        s = open(p).read()
        if old not in s:
            raise SystemExit("no match in %s: %r" % (f, old[:80]))
        open(p, "w").write(s.replace(old, new))
    out = os.path.join(REPO, "variants")
    os.makedirs(out, exist_ok=True)
    csrc = os.path.join(root, "pkg", "csrc")
    srcs = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".cpp")))
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-shared", "-munsafe-fp-atomics", "-fno-gpu-rdc", "-ffp-contract=off",
                        "-DSL_BUILD_ID=\"var-%s\"" % name, "-Rpass-analysis=kernel-resource-usage"]
                       + srcs + ["-o", os.path.join(out, name + ".so")],
                       capture_output=True, text=True)
    if r.returncode:
        sys.stderr.write(r.stderr[-4000:])
        raise SystemExit(1)
    info = {}
    fn = None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            fn = m.group(1)
        m = re.search(r"(VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and fn and "k_env_step_" in fn and "generic" not in fn:
            info.setdefault(fn, {})[m.group(1).split()[0] + ("sp" if "Spill" in m.group(1) and "S" == m.group(1)[0] and "SGPR" in m.group(1) else ("vsp" if "Spill" in m.group(1) else ""))] = m.group(2)
    for fn, d in info.items():
        k = re.search(r"k_env_step_[a-z0-9]+(I\w*?E)?(?=E|N|v)", fn)
        print("%-14s %-34s %s" % (name, k.group(0) if k else fn[-30:], " ".join("%s=%s" % kv for kv in sorted(d.items()))))

if __name__ == "__main__":
    if len(sys.argv) < 2:
        raise SystemExit(__doc__)
    ns = {}
    exec(open(sys.argv[1]).read(), ns)
    for n, reps in ns["VARIANTS"].items():
        if len(sys.argv) == 2 or n in sys.argv[2:]:
            main(n, reps)
