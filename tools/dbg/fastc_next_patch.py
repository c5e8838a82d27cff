# Build-variant edit: the coalesced kernel's next chunk index computed
# incrementally (the run's next chunk, or the next run kRunC * nw chunks on)
# instead of chunk_of's 64-bit multiply per iteration; the same values,
# capped at nchunks the same way.
t = s
a = """  for (;;) {
    const uint32_t cn = chunk_of(kth + 1);
    u32x4 nxt[4];"""
assert a in t
t = t.replace(a, """  for (;;) {
    // == chunk_of(kth + 1): within a run the next chunk, after a run's last
    // the first of the wave's next run (kRunC * nw chunks on)
    const uint32_t cu = (kth + 1u) % kRunC ? c + 1u : c + 1u - kRunC + kRunC * nw;
    const uint32_t cn = cu < nchunks ? cu : nchunks;
    u32x4 nxt[4];""", 1)
out = t
