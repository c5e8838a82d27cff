# Build-variant edit (VFILE=ixgrx_ev.hip): ixg_ev_count takes its chunks 4 at
# a time, all record / demux loads issued before the first ballot (the loop
# waited for one chunk's loads per iteration: ~100 us for 16M records).
t = s
a = """  for (uint32_t k = 0, c = ev_chunk(0, nw, nchunks); c < nchunks; c = ev_chunk(++k, nw, nchunks)) {
    const Ev e = classify(p, c * 64u + (uint32_t)lane);
    const uint64_t m = __ballot(e.on);
    if (lane == 0) p.chunk_base[c] = (uint32_t)__popcll(m);
  }"""
assert a in t
t = t.replace(a, """  // four chunks per step: their loads are all in flight before the first
  // ballot (a chunk past the end classifies as empty and stores nothing)
  constexpr uint32_t U = 4;
  for (uint32_t k = 0;; k += U) {
    uint32_t cs[U];
    bool on[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      cs[u] = ev_chunk(k + u, nw, nchunks);
      on[u] = classify(p, cs[u] * 64u + (uint32_t)lane).on;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint64_t m = __ballot(on[u]);
      if (lane == 0 && cs[u] < nchunks) p.chunk_base[cs[u]] = (uint32_t)__popcll(m);
    }
    if (cs[U - 1] >= nchunks) break;
  }""", 1)
out = t
