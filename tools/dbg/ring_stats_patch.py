# Build-variant edit (tools/build_variant.sh): the ring kernel with cycle
# counters (s_memtime) per block; read back by tools/dbg/ring_stats.py.
t = s
def rep(a, b):
    global t
    assert a in t, a[:60]
    t = t.replace(a, b, 1)
rep("typedef __attribute__((address_space(3))) RingQ lds_ringq;",
    "typedef __attribute__((address_space(3))) RingQ lds_ringq;\n"
    "__device__ unsigned long long g_ring_stats[16];\n"
    "#define RST(k, v) atomicAdd(&g_ring_stats[k], (unsigned long long)(v))\n")
# loader: total, blocked-on-room cycles, header-wait cycles, blocked iterations
rep("  uint32_t vpos = 0, vhdr = 0, vend = 0;",
    "  uint32_t vpos = 0, vhdr = 0, vend = 0;\n  uint64_t tl0 = __builtin_amdgcn_s_memtime(), tblk = 0, thdr = 0, nblk = 0;")
rep("      wait_for(rl(vhdr, s));",
    "      { uint64_t a_ = __builtin_amdgcn_s_memtime(); wait_for(rl(vhdr, s)); thdr += __builtin_amdgcn_s_memtime() - a_; }")
rep("    // room: at most kRingQ entries, and the slots behind the oldest entry in use\n    for (;;) {\n      advance();",
    "    // room: at most kRingQ entries, and the slots behind the oldest entry in use\n    uint64_t b_ = __builtin_amdgcn_s_memtime();\n    for (;;) {\n      advance();")
rep("""      if (s - old < kRingQ && pos + npc - base <= NS) break;""",
    """      if (s - old < kRingQ && pos + npc - base <= NS) break;\n      nblk++;""")
rep("""    const uint32_t e_ = s % kRingQ;
    if (li == 0u) {""", """    tblk += __builtin_amdgcn_s_memtime() - b_;
    const uint32_t e_ = s % kRingQ;
    if (li == 0u) {""")
rep("""  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
  landed = issued;
  publish();
}
""", """  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
  landed = issued;
  publish();
  if (lane == 0) { RST(0, __builtin_amdgcn_s_memtime() - tl0); RST(1, tblk); RST(2, thdr); RST(3, nblk); RST(10, 1); }
}
""")
# consumer: ready wait, phase R, phase P, chunks
rep("""  bool deferred = false;
  for (;;) {
    uint32_t t = 0;""", """  bool deferred = false;
  uint64_t trd = 0, tR = 0, tP = 0, nch = 0, tw0 = __builtin_amdgcn_s_memtime();
  for (;;) {
    uint32_t t = 0;""")
rep("""    for (int l = 0; l < kRingLoaders; l++)
      while (lds_load(&q->ready[l][e]) != t + 1u) __builtin_amdgcn_s_sleep(1);""",
    """    uint64_t r0_ = __builtin_amdgcn_s_memtime();
    for (int l = 0; l < kRingLoaders; l++)
      while (lds_load(&q->ready[l][e]) != t + 1u) __builtin_amdgcn_s_sleep(1);
    uint64_t r1_ = __builtin_amdgcn_s_memtime(); trd += r1_ - r0_; nch++;""")
rep("""    // ---- phase P: parse, records ----""", """    uint64_t r2_ = __builtin_amdgcn_s_memtime(); tR += r2_ - r1_;
    // ---- phase P: parse, records ----""")
rep("""      store_demux<DMX>(p, i, r, st.src, st.dst, st.ports);
    }
  }
  return deferred;""", """      store_demux<DMX>(p, i, r, st.src, st.dst, st.ports);
    }
    tP += __builtin_amdgcn_s_memtime() - r2_;
  }
  if (lane == 0) { RST(4, trd); RST(5, tR); RST(6, tP); RST(7, nch); RST(8, __builtin_amdgcn_s_memtime() - tw0); RST(9, 1); }
  return deferred;""")
rep("""extern "C" uint32_t ixgrx_kparams_size(void)""", """extern "C" int ixgrx_ring_stats(unsigned long long* out, int reset) {
  hipDeviceSynchronize();
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ring_stats), sizeof(g_ring_stats)) != hipSuccess) return -1;
  if (reset) { unsigned long long z[16] = {0}; hipMemcpyToSymbol(HIP_SYMBOL(g_ring_stats), z, sizeof(z)); }
  return 0;
}
extern "C" uint32_t ixgrx_kparams_size(void)""")
out = t
# phase R sub-phases: header + inside check, prefix + edges, tail rounds
t = t.replace("    const uint32_t ra = wrap((pos % NS) * 1024u + (valid ? (uint32_t)rel64 : 0u));",
              "    const uint32_t ra = wrap((pos % NS) * 1024u + (valid ? (uint32_t)rel64 : 0u));\n"
              "    uint64_t s1_ = __builtin_amdgcn_s_memtime(); tH_ += s1_ - r1_;", 1)
t = t.replace("    // whole pieces [a16, e16): medium segments (<= 32 pieces) by 4-lane",
              "    uint64_t s2_ = __builtin_amdgcn_s_memtime(); tPE_ += s2_ - s1_;\n"
              "    // whole pieces [a16, e16): medium segments (<= 32 pieces) by 4-lane", 1)
t = t.replace("    const uint32_t tail = npi ? add1c(edge, ws[lane]) : edge;",
              "    const uint32_t tail = npi ? add1c(edge, ws[lane]) : edge;\n"
              "    tT_ += __builtin_amdgcn_s_memtime() - s2_;", 1)
t = t.replace("  uint64_t trd = 0, tR = 0, tP = 0, nch = 0, tw0 = __builtin_amdgcn_s_memtime();",
              "  uint64_t trd = 0, tR = 0, tP = 0, nch = 0, tw0 = __builtin_amdgcn_s_memtime(), tH_ = 0, tPE_ = 0, tT_ = 0;", 1)
t = t.replace("RST(8, __builtin_amdgcn_s_memtime() - tw0); RST(9, 1); }",
              "RST(8, __builtin_amdgcn_s_memtime() - tw0); RST(9, 1); RST(11, tH_); RST(12, tPE_); RST(13, tT_); }", 1)
out = t
