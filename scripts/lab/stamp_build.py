#!/usr/bin/env python3
"""Lab build: sheep_kernels.hip with per-phase clock stamps in the front-half kernels.

Copies the library sources to a scratch directory, inserts a stamp after every block_sync()
(and at the end) of the kernels named on the command line, and builds
sheep_amd/libsheep_amd_lab.so.  Thread 0 of each block adds the shader clocks since its previous
stamp to g_lab[16 * kid + i] (i: the stamp's running index in that block); sheep_lab_stamps()
(appended to the copy only) reads and clears them.  The product sources are not touched.

    python scripts/lab/stamp_build.py k_front_fused k_edge_bin k_part
"""
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "sheep_amd", "csrc")

HEAD = r'''
__device__ unsigned long long g_lab[256];
#define LAB_BEGIN unsigned long long lab_t = clock64(); uint32_t lab_i = 0;
#define LAB_STAMP(kid) do { if (threadIdx.x == 0) { const unsigned long long lab_n = clock64(); \
  atomicAdd(&g_lab[16 * (kid) + min(lab_i, 15u)], lab_n - lab_t); lab_t = lab_n; } ++lab_i; } while (0)
'''

TAIL = r'''
extern "C" int sheep_lab_stamps(unsigned long long* out, int n) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sheep::g_lab), (size_t)n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  static unsigned long long zero[256];
  return hipMemcpyToSymbol(HIP_SYMBOL(sheep::g_lab), zero, sizeof(zero), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
'''


def instrument(src, name, kid):
    m = re.search(r"\n(k_%s|%s)\(" % (re.escape(name[2:]), re.escape(name)), src)
    if not m:
        raise SystemExit("kernel %s not found" % name)
    i = src.index("{", m.end())  # the body's opening brace (after the parameter list)
    depth, j = 0, i
    while True:
        c = src[j]
        if c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                break
        j += 1
    body = src[i + 1:j]
    body = body.replace("block_sync();", "block_sync(); LAB_STAMP(%d);" % kid)
    return src[:i + 1] + " LAB_BEGIN " + body + " LAB_STAMP(%d); " % kid + src[j:]


def main():
    names = sys.argv[1:] or ["k_front_fused", "k_edge_bin", "k_part"]
    out = os.path.join(ROOT, "sheep_amd", "csrc_lab")  # (beside csrc: its relative includes hold)
    shutil.rmtree(out, ignore_errors=True)
    shutil.copytree(CSRC, out)
    p = os.path.join(out, "sheep_kernels.hip")
    src = open(p).read()
    anchor = "static constexpr uint32_t FAULT_STEPS"
    src = src.replace(anchor, HEAD + anchor, 1)
    for kid, n in enumerate(names):
        src = instrument(src, n, kid)
    src += TAIL
    open(p, "w").write(src)
    lab = os.path.join(ROOT, "sheep_amd", "libsheep_amd_lab.so")
    subprocess.run(["make", "-s", "-C", out, "OUT=" + lab], check=True)
    print("built", lab, "kernels:", ", ".join("%d=%s" % (k, n) for k, n in enumerate(names)))


if __name__ == "__main__":
    main()
