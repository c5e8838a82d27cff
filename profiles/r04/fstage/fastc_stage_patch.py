# Build-variant edit: the coalesced kernel issues its hash-table loads, then
# its first chunk's frame loads, and only then writes the tables to LDS and
# joins the block barrier, so each block's first chunk is in flight during
# the table staging (8 blocks per CU slot per launch each paid the staging
# latency before their first frame load).
t = s
# 1. the kernels no longer stage before the loop
for k in ("ixg_rx_fastc_s", "ixg_rx_fastc_dmx_s"):
    a = k + "(KParams p) {\n  __shared__ uint64_t T[12 * 256];\n  __shared__ uint32_t buf[kWaves][1024];\n  stage_tables(p, T);\n"
    assert a in t, k
    t = t.replace(a, k + "(KParams p) {\n  __shared__ uint64_t T[12 * 256];\n  __shared__ uint32_t buf[kWaves][1024];\n", 1)
t = t.replace("fastc_loop<false>(p, T, LDS(lds_u32, buf[threadIdx.x >> 6]));",
              "fastc_loop<false>(p, T, T, LDS(lds_u32, buf[threadIdx.x >> 6]));")
t = t.replace("fastc_loop<true>(p, T, LDS(lds_u32, buf[threadIdx.x >> 6]));",
              "fastc_loop<true>(p, T, T, LDS(lds_u32, buf[threadIdx.x >> 6]));")
# 2. the loop stages them after the first issue
a = "DEV void fastc_loop(const KParams& p, const uint64_t* __restrict__ T, lds_u32* buf) {"
assert a in t
t = t.replace(a, "DEV void fastc_loop(const KParams& p, const uint64_t* __restrict__ T, uint64_t* Tw, lds_u32* buf) {", 1)
a = """  uint32_t c = chunk_of(0);
  if (c >= nchunks) return;
  uint64_t dmask = 0;"""
assert a in t
t = t.replace(a, """  uint32_t c = chunk_of(0);
  constexpr int kTabV = 12 * 256 / 2 / kBlock;
  static_assert(kTabV * kBlock == 12 * 256 / 2, "table pieces per thread");
  uint64_t dmask = 0;""", 1)
a = """  fastc_issue(p, c, nchunks, lim, lane, cur, Lc);
  for (;;) {"""
assert a in t
t = t.replace(a, """  u32x4 tv[kTabV];
#pragma unroll
  for (int k = 0; k < kTabV; k++) tv[k] = reinterpret_cast<const u32x4*>(p.tab)[threadIdx.x + k * kBlock];
  fastc_issue(p, c, nchunks, lim, lane, cur, Lc);
#pragma unroll
  for (int k = 0; k < kTabV; k++) reinterpret_cast<u32x4*>(Tw)[threadIdx.x + k * kBlock] = tv[k];
  __syncthreads();
  if (c >= nchunks) return;
  for (;;) {""", 1)
out = t
