#!/usr/bin/env python3
"""Build libsafelife_hip.so from the sources of a git revision, optionally patched
(A/B timing against an earlier kernel): build_rev.py <rev> <name> [spec.py variant]

The revision's safelife-k2_amd/csrc and include/ are exported to /tmp/slrev/<name>,
the literal replacements of VARIANTS[variant] in spec.py (tools/build_variant.py's
format) are applied, and the library is built with the shipped flags into
variants/<name>.so (git-ignored; load it with SAFELIFE_HIP_LIB=variants/<name>.so).
"""
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(rev, name, spec=None, variant=None):
    root = os.path.join("/tmp/slrev", name)
    shutil.rmtree(root, ignore_errors=True)
    os.makedirs(root)
    tar = subprocess.check_output(["git", "-C", REPO, "archive", rev, "safelife-k2_amd/csrc",
                                   "include"])
    subprocess.run(["tar", "-x", "-C", root], input=tar, check=True)
    csrc = os.path.join(root, "safelife-k2_amd", "csrc")
    if spec:
        ns = {}
        exec(open(spec).read(), ns)
        for f, old, new in ns["VARIANTS"][variant]:
            p = os.path.join(csrc, f)
            s = open(p).read()
            if old not in s:
                raise SystemExit("no match in %s: %r" % (f, old[:80]))
            open(p, "w").write(s.replace(old, new))
    out = os.path.join(REPO, "variants")
    os.makedirs(out, exist_ok=True)
    srcs = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".cpp")))
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "-fPIC", "-shared", "-munsafe-fp-atomics", "-fno-gpu-rdc",
                           "-ffp-contract=off", "-DSL_BUILD_ID=\"rev-%s\"" % name] + srcs +
                          ["-o", os.path.join(out, name + ".so")])
    print("variants/%s.so" % name)


if __name__ == "__main__":
    if len(sys.argv) < 3:
        raise SystemExit(__doc__)
    main(*sys.argv[1:5])
