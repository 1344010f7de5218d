#!/usr/bin/env python3
"""Lab build: k_kb_map with clock stamps at four points of its chunk loop (round 6 analysis).

Copies the library sources to sheep_amd/csrc_lab, and in k_kb_map adds the shader clocks of
thread 0 of each block since its previous stamp to g_lab[16 * HUB + i]:
  0 setup (before the chunk loop), 1 the wait for the chunk's records (an explicit vmcnt(0)
  after the copy from the prefetch registers), 2 classification, marks and counts up to the
  first barrier, 3 the reservation, the prefetch issue and the window flush up to the second
  barrier, 4 the kept-pair writes up to the next chunk.
Builds sheep_amd/libsheep_amd_lab.so; read with scripts/lab/stamps.py --names map map_hub.
The product sources are not touched.
"""
import os
import re
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "sheep_amd", "csrc")
HEAD = r'''
__device__ unsigned long long g_lab[256];
#define LAB_AT(kid, idx) do { if (threadIdx.x == 0) { const unsigned long long lab_n = clock64(); \
  atomicAdd(&g_lab[16 * (kid) + (idx)], lab_n - lab_t); lab_t = lab_n; } } while (0)
'''
TAIL = r'''
extern "C" int sheep_lab_stamps(unsigned long long* out, int n) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sheep::g_lab), (size_t)n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  static unsigned long long zero[256];
  return hipMemcpyToSymbol(HIP_SYMBOL(sheep::g_lab), zero, sizeof(zero), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
'''


def sub1(src, a, b):
    assert src.count(a) == 1, a
    return src.replace(a, b)


def main():
    out = os.path.join(ROOT, "sheep_amd", "csrc_lab")
    shutil.rmtree(out, ignore_errors=True)
    shutil.copytree(CSRC, out)
    p = os.path.join(out, "sheep_kernels.hip")
    src = open(p).read()
    anchor = "static constexpr uint32_t FAULT_STEPS"
    src = src.replace(anchor, HEAD + anchor, 1)
    src = sub1(src, "  if (DF >= 0) defer = DF;  // (compile-time for the one-GPU loop's deferred misses)\n",
               "  if (DF >= 0) defer = DF;  // (compile-time for the one-GPU loop's deferred misses)\n"
               "  unsigned long long lab_t = clock64();\n")
    src = sub1(src, "  uint32_t since_flush = 0;\n  for (uint32_t j = j0; j < j1; ++j) {\n",
               "  uint32_t since_flush = 0;\n  LAB_AT(HUB, 0);\n  for (uint32_t j = j0; j < j1; ++j) {\n"
               "    LAB_AT(HUB, 4);\n")
    src = sub1(src, "      vmask |= (uint32_t)(idx < c1) << r;\n    }\n",
               "      vmask |= (uint32_t)(idx < c1) << r;\n    }\n"
               "    { uint64_t lab_x = 0; for (int r = 0; r < R; ++r) lab_x ^= it[r];\n"
               "      asm volatile(\"s_waitcnt vmcnt(0)\" : : \"v\"(lab_x) : \"memory\"); }\n"
               "    LAB_AT(HUB, 1);\n")
    src = sub1(src, "    block_sync();\n    // compaction: one reservation per chunk",
               "    block_sync();\n    LAB_AT(HUB, 2);\n    // compaction: one reservation per chunk")
    src = sub1(src, "    block_sync();\n    uint32_t pos = woff[KM_THREADS / 64] + woff[w];",
               "    block_sync();\n    LAB_AT(HUB, 3);\n    uint32_t pos = woff[KM_THREADS / 64] + woff[w];")
    src += TAIL
    open(p, "w").write(src)
    lab = os.path.join(ROOT, "sheep_amd", "libsheep_amd_lab.so")
    subprocess.run(["make", "-s", "-C", out, "OUT=" + lab], check=True)
    print("built", lab)


if __name__ == "__main__":
    main()
