# Build-variant edit: a big chunk's last streaming slot issues the NEXT big
# chunk's round 0 (instead of a dummy round 16), so that round is in flight
# while the current chunk is parsed from its stash; the next chunk then
# starts with its round 0 already issued. The frame offset rides in the
# round's registers, so big_finish no longer reads the LDS descriptors that
# the next chunk's are written over.
t = s


def rep(a, b):
    global t
    assert a in t, a[:80]
    t = t.replace(a, b, 1)


rep("""  u32x4 ve;       // big rounds: the piece holding the frame end (group lane 0)
};""", """  u32x4 ve;       // big rounds: the piece holding the frame end (group lane 0)
  uint64_t boff;  // big rounds: the owner frame's offset
};""")
rep("""  const uint64_t off = ((uint64_t)w.offhi[owner] << 32) | w.offlo[owner];
  const uint8_t* f = p.base + off;
  const uint8_t* zero = p.zero + 16 * lane;
  // whole pieces only""", """  const uint64_t off = ((uint64_t)w.offhi[owner] << 32) | w.offlo[owner];
  b.boff = off;
  const uint8_t* f = p.base + off;
  const uint8_t* zero = p.zero + 16 * lane;
  // whole pieces only""")
rep("""    const uint32_t owner = b.owner < 64u ? b.owner : 0u;
    const uint64_t off = ((uint64_t)w.offhi[owner] << 32) | w.offlo[owner];
    const uint8_t* zero = p.zero + 16 * lane;""", """    const uint64_t off = b.boff;
    const uint8_t* zero = p.zero + 16 * lane;""")
rep("""template <bool OFFS, bool DMX = true>
DEV void big_chunk(const KParams& p, const uint64_t* __restrict__ T, uint32_t chunk, int lane, const WaveLds& w,
                   const GDesc& g) {
  const uint32_t i = chunk * 64u + (uint32_t)lane;
  const bool valid = i < p.n;
  const uint32_t L = g.L;  // 0 past the end
  w.end[lane] = L;
  w.offlo[lane] = (uint32_t)g.off;
  w.offhi[lane] = (uint32_t)(g.off >> 32);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  constexpr uint32_t R = 64 / kRoundPk;
  Round A, B;
  big_issue(p, w, 0, lane, A);
#pragma clang loop unroll(disable)
  for (uint32_t r = 0; r < R; r += 2) {
    big_issue(p, w, r + 1, lane, B);
    big_finish(p, w, lane, A);
    big_issue(p, w, r + 2, lane, A);
    big_finish(p, w, lane, B);
  }""", """DEV void big_descs(const WaveLds& w, int lane, uint32_t L, uint64_t off) {
  w.end[lane] = L;
  w.offlo[lane] = (uint32_t)off;
  w.offhi[lane] = (uint32_t)(off >> 32);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool OFFS, bool DMX = true>
DEV void big_chunk(const KParams& p, const uint64_t* __restrict__ T, uint32_t chunk, int lane, const WaveLds& w,
                   const GDesc& g, Round& A, bool& carried, const GDesc* Dn) {
  const uint32_t i = chunk * 64u + (uint32_t)lane;
  const bool valid = i < p.n;
  const uint32_t L = g.L;  // 0 past the end
  constexpr uint32_t R = 64 / kRoundPk;
  Round B;
  // round 0 is in flight already when the previous chunk carried it
  if (!carried) {
    big_descs(w, lane, L, g.off);
    big_issue(p, w, 0, lane, A);
  }
  // the next chunk's round 0 goes in the last slot when it is big too
  const bool carry = Dn != nullptr && wave_all(Dn->L >= kBigMin || Dn->L == 0u) && wave_any(Dn->L != 0u);
#pragma clang loop unroll(disable)
  for (uint32_t r = 0; r < R; r += 2) {
    big_issue(p, w, r + 1, lane, B);
    big_finish(p, w, lane, A);
    if (r + 2 < R) {
      big_issue(p, w, r + 2, lane, A);
    } else if (carry) {
      big_descs(w, lane, Dn->L, Dn->off);
      big_issue(p, w, 0, lane, A);
    }
    big_finish(p, w, lane, B);
  }
  carried = carry;""")
rep("""template <bool OFFS, int MODE, bool BIG, int SM = 0, bool LATE = false, bool DMX = true>
DEV bool general_chunk(const KParams& p, const uint64_t* __restrict__ T, uint32_t chunk, int lane,
                       const WaveLds& w, const GDesc& g, const GPre& x, const GDesc* Dn = nullptr,
                       GPre* Pn = nullptr) {""", """template <bool OFFS, int MODE, bool BIG, int SM = 0, bool LATE = false, bool DMX = true>
DEV bool general_chunk(const KParams& p, const uint64_t* __restrict__ T, uint32_t chunk, int lane,
                       const WaveLds& w, const GDesc& g, const GPre& x, const GDesc* Dn = nullptr,
                       GPre* Pn = nullptr, Round* carryR = nullptr, bool* carried = nullptr) {""")
rep("""    big_chunk<OFFS, DMX>(p, T, chunk, lane, w, g);""", """    big_chunk<OFFS, DMX>(p, T, chunk, lane, w, g, *carryR, *carried, Dn);""")
rep("""  for (uint32_t j = 0; j < nq; j++) {
    const uint32_t c2 = j + 2 < nq ? q[j + 2] : kNoChunk;
    GDesc D2;
    gen_desc<OFFS>(p, c2, lane, D2);
    GPre P1;
    if (EARLY) gen_pre<GATE, BIG>(p, D1, lane, P1);
    constexpr bool LATE = LATE_OK && !EARLY && MODE == kModeLong;
    deferred |= general_chunk<OFFS, MODE, BIG, SM, LATE, DMX>(p, T, c0, lane, w, D0, P0, &D1, &P1);""", """  Round carryR;
  bool carried = false;
  for (uint32_t j = 0; j < nq; j++) {
    const uint32_t c2 = j + 2 < nq ? q[j + 2] : kNoChunk;
    GDesc D2;
    gen_desc<OFFS>(p, c2, lane, D2);
    GPre P1;
    if (EARLY) gen_pre<GATE, BIG>(p, D1, lane, P1);
    constexpr bool LATE = LATE_OK && !EARLY && MODE == kModeLong;
    deferred |= general_chunk<OFFS, MODE, BIG, SM, LATE, DMX>(p, T, c0, lane, w, D0, P0, &D1, &P1, &carryR,
                                                              &carried);""")
out = t
