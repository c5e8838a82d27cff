# Build-variant edit: two chunks in flight per wave with the product's two
# register sets. The product's loop issues chunk k+1 into `nxt` and copies
# `nxt` into `cur` at the end of the iteration; the compiler places the copy
# (and the wait for the data it needs) before the next loads, so a wave has
# one chunk in flight. Here each set is written to LDS, then immediately
# reloaded with the chunk two ahead, then the chunk is parsed from LDS: while
# chunk k is parsed, chunks k+1 (the other set) and k+2 (this set) are in
# flight, in the same 32 VGPRs.
import re

t = s
head = """  for (;;) {
    const uint32_t cn = chunk_of(kth + 1);
    u32x4 nxt[4];
    uint32_t Ln;
    fastc_issue(p, cn, nchunks, lim, lane, nxt, Ln);
"""
tail = """    c = cn;
    if (c >= nchunks) break;
#pragma unroll
    for (int k = 0; k < 4; k++) cur[k] = nxt[k];
    Lc = Ln;
  }
"""
a = t.index(head)
b = t.index(tail, a)
body = t[a + len(head):b]
# the LDS writes, then the set's reload with the chunk two ahead
w = """#pragma unroll
    for (int k = 0; k < 4; k++) {
      lds_u32* w = buf + 4 * (lane + 64 * k);
      w[0] = cur[k].x; w[1] = cur[k].y; w[2] = cur[k].z; w[3] = cur[k].w;
    }
"""
assert w in body
body = body.replace(w, w + """    const uint32_t Lc = Lv;
    fastc_issue(p, ca, nchunks, lim, lane, cv, Lv);
""")
body = body.replace("cur[k]", "cv[k]")
body = re.sub(r"\bc\b", "cc", body)
new = """  // (two chunks in flight: each register set goes to LDS and is reloaded
  // with the chunk two ahead before its chunk is parsed)
  u32x4 alt[4];
  uint32_t La = 0;
  uint32_t c1 = chunk_of(1);
  fastc_issue(p, c1, nchunks, lim, lane, alt, La);
  auto body = [&](u32x4 (&cv)[4], uint32_t& Lv, uint32_t cc, uint32_t ca) {
""" + body + """  };
  for (;;) {
    const uint32_t c2 = chunk_of(kth + 2);
    body(cur, Lc, c, c2);
    if (c1 >= nchunks) break;
    const uint32_t c3 = chunk_of(kth + 2);
    body(alt, La, c1, c3);
    if (c2 >= nchunks) break;
    c = c2;
    c1 = c3;
  }
"""
t = t[:a] + new + t[b + len(tail):]
out = t
