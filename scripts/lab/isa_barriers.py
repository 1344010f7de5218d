#!/usr/bin/env python3
"""Check, in gfx950 assembly, that every s_barrier of each kernel is preceded by a wait that
drains the wave's LDS operations (s_waitcnt with lgkmcnt(0)) with no LDS instruction between.

    python scripts/lab/isa_barriers.py <kernels.s>   # from hipcc --cuda-device-only -S
    python scripts/lab/isa_barriers.py --build [REV] # compile sheep_kernels.hip (at git REV) first

Used for VERDICT r02 item 5: the committed parent of fe956ff (plain __syncthreads()) already
had the wait in front of all four barriers of k_degb_hist16.
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "sheep_amd", "csrc")


def build(rev=None):
    d = tempfile.mkdtemp(prefix="isa_")
    for f in ("sheep_kernels.hip", "sheep_internal.h", "sheep_comm.h", "rmat.h", "powerlaw.h"):
        if rev:
            src = subprocess.run(["git", "-C", ROOT, "show", "%s:sheep_amd/csrc/%s" % (rev, f)],
                                 capture_output=True, text=True)
            if src.returncode:
                continue
            open(os.path.join(d, f), "w").write(src.stdout)
        else:
            open(os.path.join(d, f), "w").write(open(os.path.join(CSRC, f)).read())
    out = os.path.join(d, "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                    "--cuda-device-only", "-S", "-o", out, "-x", "hip",
                    os.path.join(d, "sheep_kernels.hip"), "-I", d,
                    "-I", os.path.join(ROOT, "include")], check=True)
    return out


def check(path):
    fn = None
    last_wait0 = False  # an lgkmcnt(0) wait since the last LDS instruction / label
    total = bad = 0
    per = {}
    for line in open(path):
        s = line.strip()
        m = re.match(r"^(_Z\S+):", s)
        if m:
            fn = m.group(1)
            last_wait0 = False
            continue
        if re.match(r"^\.LBB\S*:", s) or s.startswith("; %bb"):
            last_wait0 = False  # a join: another path may reach the barrier (checked per path
            continue            # only when the wait sits in the same block, as block_sync emits)
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        if op == "s_waitcnt" and "lgkmcnt(0)" in s:
            last_wait0 = True
        elif op.startswith("ds_"):
            last_wait0 = False
        elif op == "s_barrier":
            total += 1
            ok = last_wait0
            per.setdefault(fn, [0, 0])
            per[fn][0] += 1
            if not ok:
                bad += 1
                per[fn][1] += 1
    return total, bad, per


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--build":
        path = build(sys.argv[2] if len(sys.argv) > 2 else None)
    else:
        path = sys.argv[1]
    total, bad, per = check(path)
    for fn, (n, b) in sorted(per.items()):
        if b or "degb" in fn:
            print("%-80s barriers %3d  without lgkmcnt(0) in-block %d" % (fn[:80], n, b))
    print("total barriers %d, without an in-block lgkmcnt(0) wait %d" % (total, bad))


if __name__ == "__main__":
    main()
