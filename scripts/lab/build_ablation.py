"""Build a lab copy of libsheep_amd.so with one kernel variant (ablations: results WRONG, timing only):
    python scripts/lab/build_ablation.py NAME  -> scripts/lab/libsheep_NAME.so
Ablations patch the kernel text of a temporary copy; the product source is not touched."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "sheep_amd", "csrc")

PATCHES = {
    "base": [],
    "nt": [("      nx[r] = idx < c1 ? items[idx] : 0ull;", "      nx[r] = idx < c1 ? __builtin_nontemporal_load(&items[idx]) : 0ull;"),
           ("      if (it[r] != ~0ull) kept[pos + __popcll(bal & lt)] = it[r];", "      if (it[r] != ~0ull) __builtin_nontemporal_store(it[r], &kept[pos + __popcll(bal & lt)]);")],
    "r16": [("static constexpr int KM_CHUNK = 8192; ", "static constexpr int KM_CHUNK = 16384;")],
    "r12": [("static constexpr int KM_CHUNK = 8192; ", "static constexpr int KM_CHUNK = 12288;")],
    "r16np": [("static constexpr int KM_CHUNK = 8192; ", "static constexpr int KM_CHUNK = 16384;"),
              ("    if (more) fetch(c0 + KM_CHUNK);  // issued after the bitmap loads", "")],
    # s_memtime stamps of thread 0 per map phase, summed into the stats words (run with
    # SHEEP_TREE_STATS=1; the capi's tree_stats line then prints them)
    "stamp": [("  uint32_t since_flush = 0;\n", "  uint32_t since_flush = 0;\n  unsigned long long T0 = 0, T1 = 0, ph[7] = {0,0,0,0,0,0,0};\n"),
              ("    uint64_t it[R];\n    uint32_t vmask = 0;\n#pragma unroll\n    for (int r = 0; r < R; ++r) {\n      it[r] = nx[r];",
               "    T0 = __builtin_amdgcn_s_memtime();\n    uint64_t it[R];\n    uint32_t vmask = 0;\n#pragma unroll\n    for (int r = 0; r < R; ++r) {\n      it[r] = nx[r];"),
              ("    if (STATS) misses += (uint64_t)__popc(miss);\n",
               "    if (STATS) misses += (uint64_t)__popc(miss);\n    T1 = __builtin_amdgcn_s_memtime(); ph[0] += T1 - T0; T0 = T1;\n"),
              ("    // 3. roots -> giant (and its bit)", "    T1 = __builtin_amdgcn_s_memtime(); ph[1] += T1 - T0; T0 = T1;\n    // 3. roots -> giant (and its bit)"),
              ("    uint32_t nout = 0;\n", "    uint32_t nout = 0;\n    T1 = __builtin_amdgcn_s_memtime(); ph[2] += T1 - T0; T0 = T1;\n"),
              ("    if (lane == 0) woff[w] = nout;\n", "    if (lane == 0) woff[w] = nout;\n    T1 = __builtin_amdgcn_s_memtime(); ph[3] += T1 - T0; T0 = T1;\n"),
              ("    if (flush) {\n      since_flush = 0;", "    T1 = __builtin_amdgcn_s_memtime(); ph[4] += T1 - T0; T0 = T1;\n    if (flush) {\n      since_flush = 0;"),
              ("    // compaction: one reservation per chunk", "    T1 = __builtin_amdgcn_s_memtime(); ph[5] += T1 - T0; T0 = T1;\n    // compaction: one reservation per chunk"),
              ("    // no barrier here: the next chunk", "    T1 = __builtin_amdgcn_s_memtime(); ph[6] += T1 - T0; T0 = T1;\n    // no barrier here: the next chunk"),
              ("    atomicAdd(&stats[7], (unsigned long long)misses);\n",
               "    atomicAdd(&stats[7], (unsigned long long)misses);\n    if (t == 0) { atomicAdd(&stats[1], ph[0]); atomicAdd(&stats[2], ph[1]); atomicAdd(&stats[3], ph[2]); atomicAdd(&stats[4], ph[3]); atomicAdd(&stats[13], ph[4]); atomicAdd(&stats[14], ph[5]); atomicAdd(&stats[15], ph[6]); }\n")],
    # smaller map blocks: more chunks in flight per CU (correct results)
    "b256": [("static constexpr int KM_THREADS = 1024;", "static constexpr int KM_THREADS = 256;"),
             ("static constexpr int KM_CHUNK = 8192; ", "static constexpr int KM_CHUNK = 2048; "),
             ("static constexpr uint32_t KM_WIN = 32768;", "static constexpr uint32_t KM_WIN = 8192;"),
             ("std::min<uint64_t>(chunks, 512);", "std::min<uint64_t>(chunks, 1280);")],
    "b512": [("static constexpr int KM_THREADS = 1024;", "static constexpr int KM_THREADS = 512;"),
             ("static constexpr int KM_CHUNK = 8192; ", "static constexpr int KM_CHUNK = 4096; "),
             ("static constexpr uint32_t KM_WIN = 32768;", "static constexpr uint32_t KM_WIN = 16384;"),
             ("std::min<uint64_t>(chunks, 512);", "std::min<uint64_t>(chunks, 768);")],
    "b256w16": [("static constexpr int KM_THREADS = 1024;", "static constexpr int KM_THREADS = 256;"),
             ("static constexpr int KM_CHUNK = 8192; ", "static constexpr int KM_CHUNK = 2048; "),
             ("static constexpr uint32_t KM_WIN = 32768;", "static constexpr uint32_t KM_WIN = 16384;"),
             ("std::min<uint64_t>(chunks, 512);", "std::min<uint64_t>(chunks, 1024);")],
    # no hi counts at all (pst wrong)
    "nocnt": [("if (valid && cnt) {", "if (false) {"),
              ("    if (cnt)\n      for (uint32_t i = t; i < (span + 1) / 2; i += KM_THREADS) {\n        uint32_t v = wcnt[i];",
               "    if (false)\n      for (uint32_t i = t; i < (span + 1) / 2; i += KM_THREADS) {\n        uint32_t v = wcnt[i];")],
    # counts kept in LDS only (no global flush)
    "noflush": [("        if (v & 0xFFFFu) atomicAdd(&cnt[bbase + 2 * i], v & 0xFFFFu);\n        if (v >> 16) atomicAdd(&cnt[bbase + 2 * i + 1], v >> 16);",
                 "        if (v == 0xFFFFFFFFu) cnt[0] = v;")],
    # no kept writes
    "nokept": [("      if (it[r] != ~0ull) kept[pos + __popcll(bal & lt)] = it[r];", "      if (it[r] == 1ull) kept[0] = it[r];")],
    # no finds: every miss is taken as giant
    "nofind": [("    for (uint32_t act = miss; act;) {", "    for (uint32_t act = 0; act;) {")],
    # partition tiles: 8K records (2 blocks / CU) or 4K (4 blocks / CU)
    "pt512": [("static constexpr int PT_THREADS = 1024;", "static constexpr int PT_THREADS = 512;")],
    "pt1k8": [("static constexpr int PT_ITEMS = 16;", "static constexpr int PT_ITEMS = 8;")],
    "pt256": [("static constexpr int PT_THREADS = 1024;", "static constexpr int PT_THREADS = 256;")],
    # degree scatter chunks of 16K records (64 KB LDS: 2 blocks / CU)
    "dg16": [("static constexpr int DEGB_CHUNK = 32768;", "static constexpr int DEGB_CHUNK = 16384;")],
    # partition cursors one per 128-B line (same-line atomics from every tile)
    "ptpad": [("gbase[t] = c ? atomicAdd(&cursor[t], (unsigned long long)c) : 0ull;",
               "gbase[t] = c ? atomicAdd(&cursor[16 * t], (unsigned long long)c) : 0ull;"),
              ("  cursor[t] = s[t];\n  hist[t] = 0;", "  cursor[16 * t] = s[t];\n  hist[t] = 0;")],
    # partition without the LDS stage: each record is stored straight from registers to its
    # reserved run (order inside a run by LDS-atomic order); 3 KB of LDS -> 2 blocks / CU
    "ptdirect": [("  __shared__ uint64_t stage[PT_TILE];\n  __shared__ uint32_t hist[256], tstart[256]", "  __shared__ uint32_t hist[256], tstart[256]"),
                 ("""      stage[tstart[part_digit(key, sh)] + li[k]] = rec[k];
    }
  }
  __syncthreads();
  for (uint32_t j = t; j < tile_n; j += PT_THREADS) {
    uint64_t r = stage[j];
    uint32_t d = part_digit(MODE == 0 ? (uint32_t)(r >> 32) : (uint32_t)r, sh);
    out[gbase[d] + (j - tstart[d])] = r;
  }""", """      out[gbase[part_digit(key, sh)] + li[k]] = rec[k];
    }
  }""")],
    # partition loads of 16 B per lane (two records; lab only: assumes 16-B aligned input)
    "pt16b": [("""#pragma unroll
  for (int k = 0; k < PT_ITEMS; ++k) {
    uint32_t j = (uint32_t)k * PT_THREADS + t;
    rec[k] = j < tile_n ? in[tbase + j] : 0ull;
  }""", """#pragma unroll
  for (int k = 0; k < PT_ITEMS; k += 2) {
    uint32_t j = (uint32_t)(k >> 1) * 2 * PT_THREADS + 2 * t;
    if (j + 1 < tile_n) {
      ulonglong2 q = *(const ulonglong2*)(in + tbase + j);
      rec[k] = q.x; rec[k + 1] = q.y;
    } else {
      rec[k] = j < tile_n ? in[tbase + j] : 0ull;
      rec[k + 1] = 0ull;
    }
  }"""),
              ("""    if ((uint32_t)k * PT_THREADS + t < tile_n) {
      uint32_t key = MODE == 0 ? (uint32_t)(rec[k] >> 32) : (uint32_t)rec[k];
      li[k]""", """    if ((uint32_t)(k >> 1) * 2 * PT_THREADS + 2 * t + (k & 1) < tile_n) {
      uint32_t key = MODE == 0 ? (uint32_t)(rec[k] >> 32) : (uint32_t)rec[k];
      li[k]"""),
              ("""    if ((uint32_t)k * PT_THREADS + t < tile_n) {
      uint32_t key = MODE == 0 ? (uint32_t)(rec[k] >> 32) : (uint32_t)rec[k];
      stage""", """    if ((uint32_t)(k >> 1) * 2 * PT_THREADS + 2 * t + (k & 1) < tile_n) {
      uint32_t key = MODE == 0 ? (uint32_t)(rec[k] >> 32) : (uint32_t)rec[k];
      stage""")],
    # fewer map blocks: the concurrent apply (the critical path) gets more of the chip
    "mg256": [("std::min<uint64_t>(chunks, 512);", "std::min<uint64_t>(chunks, 256);")],
    "mg192": [("std::min<uint64_t>(chunks, 512);", "std::min<uint64_t>(chunks, 192);")],
    "mg320": [("std::min<uint64_t>(chunks, 512);", "std::min<uint64_t>(chunks, 320);")],
    "mg384": [("std::min<uint64_t>(chunks, 512);", "std::min<uint64_t>(chunks, 384);")],
    "mg128": [("std::min<uint64_t>(chunks, 512);", "std::min<uint64_t>(chunks, 128);")],
    # bin scatter tiles of 8192 items, 512 threads, 64 KB stage: two blocks per CU
    "bs512": [("static constexpr int BS_TILE = 2 * RS_TILE;", "static constexpr int BS_TILE = RS_TILE;"),
              ("__global__ void __launch_bounds__(1024)\nk_bin_scatter(", "__global__ void __launch_bounds__(512)\nk_bin_scatter("),
              ("  constexpr int NT = 1024, IT = BS_TILE / NT;\n  __shared__ uint64_t stage[BS_TILE];\n  __shared__ uint32_t hist[512], tstart[512], goff[512], wsum[NT / 64];",
               "  constexpr int NT = 512, IT = BS_TILE / NT;\n  __shared__ uint64_t stage[BS_TILE];\n  __shared__ uint32_t hist[512], tstart[512], goff[512], wsum[NT / 64];"),
              ("    goff[t] = offsets[(uint64_t)(2 * blockIdx.x) * 512 + t];\n  }\n  uint64_t it[IT];",
               "    goff[t] = offsets[(uint64_t)blockIdx.x * 512 + t];\n  }\n  uint64_t it[IT];"),
              ("dim3((unsigned)((n + BS_TILE - 1) / BS_TILE)), dim3(1024), 0, s,", "dim3((unsigned)((n + BS_TILE - 1) / BS_TILE)), dim3(512), 0, s,")],
    # zipper without the jump hints (results unchanged: hints only)
    "zipnojump": [("    tree_queue_body<0, 1, STATS, true, true>(src, src.np + nk,", "    tree_queue_body<0, 0, STATS, true, true>(src, src.np + nk,"),
                  ("    tree_queue_body<0, 1, STATS, true, false>(src, nk,", "    tree_queue_body<0, 0, STATS, true, false>(src, nk,")],
    # zipper parent loads as plain loads (L1/L2 cached) instead of agent-scope atomic loads
    "zipplain": [("  if (LOAD == 0) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);", "  if (LOAD == 0) return *(volatile uint32_t*)p;")],
    # zipper: no jump-hint load on the first step of a pending edge (most edges take one step)
    "zipj2": [("    if (JUMP) {\n      const uint32_t j = jump[s.x];", "    if (JUMP && !(s.x == s.a && s.prev == INV)) {\n      const uint32_t j = jump[s.x];")],
    # zipper grid / queue chunk
    "zg512": [("    hipLaunchKernelGGL(zk, dim3(MAX_GRID), dim3(BLOCK), 0, s, kept,", "    hipLaunchKernelGGL(zk, dim3(512), dim3(BLOCK), 0, s, kept,")],
    "zg1024": [("    hipLaunchKernelGGL(zk, dim3(MAX_GRID), dim3(BLOCK), 0, s, kept,", "    hipLaunchKernelGGL(zk, dim3(1024), dim3(BLOCK), 0, s, kept,")],
    "zq64": [("    const uint32_t qchunk = 256;", "    const uint32_t qchunk = 64;")],
    "zq512": [("    const uint32_t qchunk = 256;", "    const uint32_t qchunk = 512;")],
    # (timing-only ablations that leave buffers unwritten are NOT safe: one of them hung and
    # faulted the GPU — garbage ids reach kernels that index with them.  Keep variants exact.)
    "front": [],
    # streaming loads / stores of the edge-bin and partition passes non-temporal
    "ebinnt": [("    e[k] = j < tile_n ? uv[tbase + j] : make_uint2(0, PRE ? RY_SELF : 0u);",
                "    if (j < tile_n) { const uint64_t q = __builtin_nontemporal_load((const uint64_t*)uv + tbase + j); e[k] = make_uint2((uint32_t)q, (uint32_t)(q >> 32)); } else e[k] = make_uint2(0, PRE ? RY_SELF : 0u);")],
    "ebonnt": [("""    const uint32_t s0 = tstart[d];
    for (uint32_t j = lane; j < c; j += 64) out[g + j] = stage[s0 + j];
  }
}

void launch_edge_bin(""", """    const uint32_t s0 = tstart[d];
    for (uint32_t j = lane; j < c; j += 64) __builtin_nontemporal_store(stage[s0 + j], &out[g + j]);
  }
}

void launch_edge_bin(""")],
    "partnt": [("    rec[k] = j < tile_n ? in[tbase + j] : 0ull;", "    rec[k] = j < tile_n ? __builtin_nontemporal_load(&in[tbase + j]) : 0ull;"),
               ("    out[gbase[d] + (j - tstart[d])] = r;", "    __builtin_nontemporal_store(r, &out[gbase[d] + (j - tstart[d])]);")],
    # map record loads non-temporal (the streamed records should not evict the apply's working set)
    "mapnt": [("      nx[r] = idx < nc1 ? items[idx] : 0ull;", "      nx[r] = idx < nc1 ? __builtin_nontemporal_load(&items[idx]) : 0ull;")],
    # two map blocks per CU (for the unpipelined loop, where the map has the chip to itself)
    "mg2": [("std::min<uint64_t>(chunks, device_cus());", "std::min<uint64_t>(chunks, 2 * device_cus());")],
    # map blocks of 256 / 512 threads keeping the 32K-rank window (fewer map waves per CU beside the apply)
    "m256": [("static constexpr int KM_THREADS = 1024;", "static constexpr int KM_THREADS = 256;"),
             ("static constexpr int KM_CHUNK = 8192; ", "static constexpr int KM_CHUNK = 2048; "),
             ("std::min<uint64_t>(chunks, device_cus());", "std::min<uint64_t>(chunks, 2 * device_cus());")],
    "m512": [("static constexpr int KM_THREADS = 1024;", "static constexpr int KM_THREADS = 512;"),
             ("static constexpr int KM_CHUNK = 8192; ", "static constexpr int KM_CHUNK = 4096; "),
             ("std::min<uint64_t>(chunks, device_cus());", "std::min<uint64_t>(chunks, 2 * device_cus());")],
    "m512g1": [("static constexpr int KM_THREADS = 1024;", "static constexpr int KM_THREADS = 512;"),
             ("static constexpr int KM_CHUNK = 8192; ", "static constexpr int KM_CHUNK = 4096; ")],
    # degree kernels (correct results): loads in flight, flat write-out of the staged runs
    "h16v2": [("  uint32_t acc[64];\n#pragma unroll\n  for (int k = 0; k < 64; ++k) acc[k] = 0;\n  constexpr int V = 4;",
               "  uint32_t acc[64];\n#pragma unroll\n  for (int k = 0; k < 64; ++k) acc[k] = 0;\n  constexpr int V = 2;")],
    "h16v8": [("  uint32_t acc[64];\n#pragma unroll\n  for (int k = 0; k < 64; ++k) acc[k] = 0;\n  constexpr int V = 4;",
               "  uint32_t acc[64];\n#pragma unroll\n  for (int k = 0; k < 64; ++k) acc[k] = 0;\n  constexpr int V = 8;")],
    "dsu4": [("  const uint64_t base = (uint64_t)blockIdx.x * DEGB_CHUNK;\n  const uint32_t cn = (uint32_t)min((uint64_t)DEGB_CHUNK, m - base);\n  constexpr int U = 8;\n  for (int r = 0; r < DEGB_CHUNK / (DEGB_THREADS * U); ++r) {\n    uint2 ee[U];",
              "  const uint64_t base = (uint64_t)blockIdx.x * DEGB_CHUNK;\n  const uint32_t cn = (uint32_t)min((uint64_t)DEGB_CHUNK, m - base);\n  constexpr int U = 4;\n  for (int r = 0; r < DEGB_CHUNK / (DEGB_THREADS * U); ++r) {\n    uint2 ee[U];")],
    "dsu16": [("  const uint64_t base = (uint64_t)blockIdx.x * DEGB_CHUNK;\n  const uint32_t cn = (uint32_t)min((uint64_t)DEGB_CHUNK, m - base);\n  constexpr int U = 8;\n  for (int r = 0; r < DEGB_CHUNK / (DEGB_THREADS * U); ++r) {\n    uint2 ee[U];",
               "  const uint64_t base = (uint64_t)blockIdx.x * DEGB_CHUNK;\n  const uint32_t cn = (uint32_t)min((uint64_t)DEGB_CHUNK, m - base);\n  constexpr int U = 16;\n  for (int r = 0; r < DEGB_CHUNK / (DEGB_THREADS * U); ++r) {\n    uint2 ee[U];")],
    "dsflat": [("""  // each wave writes whole bucket runs
  for (uint32_t b = w; b < NB; b += DEGB_THREADS / 64) {
    uint32_t s0 = start[b], n = cur[b] - s0;
    uint64_t g = goff[b];
    for (uint32_t j = lane; j < n; j += 64) ep[g + j] = buf[s0 + j];
  }""", """  // flat write-out: thread t writes staged positions t, t + 1024, ...; the bucket of position
  // p is found from the bucket of position 64 (p / 64) (segment table) and a short forward scan
  __shared__ uint16_t segb[2 * DEGB_CHUNK / 64];
  for (uint32_t b = t; b < NB; b += DEGB_THREADS) {
    const uint32_t s0 = start[b], s1 = cur[b];
    for (uint32_t q = (s0 + 63) / 64; q * 64 < s1; ++q) segb[q] = (uint16_t)b;
  }
  __syncthreads();
  const uint32_t total = cur[NB - 1];
  for (uint32_t p = t; p < total; p += DEGB_THREADS) {
    uint32_t b = segb[p >> 6];
    while (cur[b] <= p) ++b;
    ep[goff[b] + (p - start[b])] = buf[p];
  }""")],
    "p1k8": [("static constexpr int PT0_THREADS = 1024, PT1_THREADS = 512;\nstatic constexpr int PT0_ITEMS = PT_ITEMS, PT1_ITEMS = PT_ITEMS;",
              "static constexpr int PT0_THREADS = 1024, PT1_THREADS = 1024;\nstatic constexpr int PT0_ITEMS = PT_ITEMS, PT1_ITEMS = 8;")],
    "p0k8": [("static constexpr int PT0_THREADS = 1024, PT1_THREADS = 512;\nstatic constexpr int PT0_ITEMS = PT_ITEMS, PT1_ITEMS = PT_ITEMS;",
              "static constexpr int PT0_THREADS = 1024, PT1_THREADS = 512;\nstatic constexpr int PT0_ITEMS = 8, PT1_ITEMS = PT_ITEMS;")],
    "p01k8": [("static constexpr int PT0_THREADS = 1024, PT1_THREADS = 512;\nstatic constexpr int PT0_ITEMS = PT_ITEMS, PT1_ITEMS = PT_ITEMS;",
               "static constexpr int PT0_THREADS = 1024, PT1_THREADS = 1024;\nstatic constexpr int PT0_ITEMS = 8, PT1_ITEMS = 8;")],
    # second partition pass writing each tile's digit-sorted stage to the tile's own range
    # (contiguous stores; the records stay exact, only their order changes) — with / without the
    # cursor atomics: what the scattered runs and the reservations cost
    "p1local": [("    out[gbase[d] + (j - tstart[d])] = r;", "    out[MODE == 1 ? tbase + j : gbase[d] + (j - tstart[d])] = r;")],
    "p1noat": [("    out[gbase[d] + (j - tstart[d])] = r;", "    out[MODE == 1 ? tbase + j : gbase[d] + (j - tstart[d])] = r;"),
               ("    gbase[t] = c ? atomicAdd(&cursor[t], (unsigned long long)c) : 0ull;",
                "    gbase[t] = (MODE == 1 || !c) ? 0ull : atomicAdd(&cursor[t], (unsigned long long)c);")],
    # (stats only, tree_stats=2) records with lo < B0, and those whose 64-rank block of the
    # giant bitmap is all ones (what a per-block summary would answer without an L2 request)
    "gsumstat": [("    if (STATS) misses += (uint64_t)__popc(miss);\n",
                  "    if (STATS) misses += (uint64_t)__popc(miss);\n"
                  "    if (STATS && use_bm) {\n"
                  "      unsigned long long c13 = 0, c14 = 0;\n"
                  "      for (int r = 0; r < R; ++r) {\n"
                  "        const uint32_t a = (uint32_t)it[r];\n"
                  "        if (((vmask >> r) & 1) && a < B0) {\n"
                  "          ++c14;\n"
                  "          if (gbits[(a >> 6) * 2] == ~0u && gbits[(a >> 6) * 2 + 1] == ~0u) ++c13;\n"
                  "        }\n"
                  "      }\n"
                  "      if (c13) atomicAdd(&stats[13], c13);\n"
                  "      if (c14) atomicAdd(&stats[14], c14);\n"
                  "    }\n"),
                 ],
    # the zipper's LDS buffer of linked roots at 2048 entries (8 KB) instead of 512
    "lcap2048": [("  constexpr uint32_t LCAP = 512;", "  constexpr uint32_t LCAP = 2048;")],
    # map grids of 3/4 and 1/2 of the CUs (with the LDS giant summary the map needs fewer
    # L2 requests; fewer map blocks leave more of the chip to the apply beside it)
    "mg34": [("std::min<uint64_t>(chunks, device_cus());", "std::min<uint64_t>(chunks, device_cus() * 3 / 4);")],
    "mgh": [("std::min<uint64_t>(chunks, device_cus());", "std::min<uint64_t>(chunks, device_cus() / 2);")],
    # hi counts: runs of equal hi in consecutive lanes added once by the run's first lane
    "cntrun": [("""      if (valid && cnt) {
        if (o < span) atomicAdd(&wcnt[o >> 1], 1u << (16 * (o & 1)));
        else atomicAdd(&cnt[b], 1u);
      }""", """      {
        const uint32_t bk = valid ? b : INV;
        const uint32_t bp = (uint32_t)__shfl_up((int)bk, 1);
        const bool lead = valid && (lane == 0 || bp != bk);
        const uint64_t brk = __ballot(!valid || lead);
        const uint64_t after = lane == 63 ? 0ull : (brk >> (lane + 1));
        const uint32_t len = after ? (uint32_t)__ffsll((unsigned long long)after) : (uint32_t)(64 - lane);
        if (lead && cnt) {
          if (o < span) atomicAdd(&wcnt[o >> 1], len << (16 * (o & 1)));
          else atomicAdd(&cnt[b], len);
        }
      }""")],
    # 64K-id histogram: leader matching only in the long (hub) runs, plain adds elsewhere
    "h16hot": [("""  uint32_t acc[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) acc[k] = 0;
  constexpr int V = 4;
  for (uint64_t g0 = s0; g0 < s1; g0 += 65535) {""", """  uint32_t acc[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) acc[k] = 0;
  constexpr int V = 4;
  if (bstart && (s1 - s0) * NB > 4 * bstart[NB]) plain = 0;  // a run 4x the mean: a hub's
  for (uint64_t g0 = s0; g0 < s1; g0 += 65535) {""")],
    # first partition pass by 512 / 2048 y digits (512 KB / 128 KB rank slices; correct results)
    "py512": [("static constexpr uint32_t PD_Y = 1024,", "static constexpr uint32_t PD_Y = 512,")],
    "eb1024x4": [("  constexpr int NT = 1024, IT = 8;", "  constexpr int NT = 1024, IT = 4;")],
    "eb1024x6": [("  constexpr int NT = 1024, IT = 8;", "  constexpr int NT = 1024, IT = 6;")],
}
CAPI_PATCHES = {
    "gsumstat": [("k, bk[k].first, bk[k + 1].first, h[0], h[5], h[6], h[7], h[8], h[9], h[10], h[11], h[12]);",
                  "k, bk[k].first, bk[k + 1].first, h[0], h[5], h[6], h[7], h[8], h[9], h[10], h[11], h[12]);\n        fprintf(stderr, \"  gsum lo<B0 %llu in-full-blocks %llu\\n\", h[14], h[13]);")],
    "front": [('    if (tm) tm->mark("edge_pass");\n    HIP_CHECK(hipEventSynchronize(c.bins_ev));',
               '    if (tm) tm->mark("edge_pass");\n    HIP_CHECK(hipEventSynchronize(c.bins_ev));\n    HIP_CHECK(hipStreamSynchronize(s));\n    if (tm) tm->mark("bin_scatter");\n    return;')],
    "ptpad": [('c.scratch.get("part_ws", 1024 * 4)', 'c.scratch.get("part_ws", 16384 * 4)')],
}


def main():
    name = sys.argv[1]
    text = open(os.path.join(SRC, "sheep_kernels.hip")).read()
    for part in name.split("+"):
        for a, b in PATCHES.get(part, []):
            assert a in text, a
            text = text.replace(a, b)
    capi = open(os.path.join(SRC, "sheep_capi.cpp")).read()
    if name == "stamp":
        a = 'h[0], h[5], h[7], h[8], h[9], h[10], h[11], h[12]);'
        assert a in capi
        capi = capi.replace(a, a + '\n    fprintf(stderr, "map_phases_cycles load+bits %llu finds %llu label %llu lds %llu barA %llu flush %llu compact+barB+write %llu\\n", h[1], h[2], h[3], h[4], h[13], h[14], h[15]);')
    for part in name.split("+"):
        for a, b in CAPI_PATCHES.get(part, []):
            assert a in capi, a
            capi = capi.replace(a, b)
    tmp = "/tmp/sheep_lab_%s" % name
    os.makedirs(tmp, exist_ok=True)
    for f in ("powerlaw.h", "rmat.h", "sheep_internal.h", "sheep_comm.h"):
        open(os.path.join(tmp, f), "w").write(open(os.path.join(SRC, f)).read())
    open(os.path.join(tmp, "sheep_kernels.hip"), "w").write(text)
    open(os.path.join(tmp, "sheep_capi.cpp"), "w").write(capi.replace('"../../include/sheep_amd.h"', '"%s"' % os.path.join(ROOT, "include", "sheep_amd.h")))
    out = os.path.join(ROOT, "scripts", "lab", "libsheep_%s.so" % name)
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall",
           "-Wno-unused-result", "-shared", "-o", out, "-I", SRC, "-x", "hip",
           os.path.join(tmp, "sheep_kernels.hip"), "-x", "hip", os.path.join(SRC, "sheep_eval.hip"),
           "-x", "hip", os.path.join(tmp, "sheep_capi.cpp"), "-x", "hip",
           os.path.join(SRC, "sheep_host.cpp"), "-x", "hip", os.path.join(SRC, "sheep_comm.cpp"), "-ldl"]
    subprocess.run(cmd, check=True)
    print(out)


if __name__ == "__main__":
    main()
