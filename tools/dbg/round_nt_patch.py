# Build-variant edit: the long kernel's streaming-round loads (round_issue,
# big_issue) non-temporal, as the span kernel's copies are (each tail piece
# is read once).
t = s
t = t.replace("""DEV u32x4 load16(bool ok, const uint8_t* addr, const uint8_t* dummy) {
  return *reinterpret_cast<const u32x4_a4*>(ok ? addr : dummy);
}""", """DEV u32x4 load16(bool ok, const uint8_t* addr, const uint8_t* dummy) {
  return *reinterpret_cast<const u32x4_a4*>(ok ? addr : dummy);
}
DEV u32x4 load16nt(bool ok, const uint8_t* addr, const uint8_t* dummy) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4_a4*>(ok ? addr : dummy));
}""", 1)
for a in ("    b.v[t] = load16(pos < b.end, f + pos, zero);",
          "    b.v[t] = load16(pos < whole, f + pos, zero);",
          "  b.ve = load16(gl == 0 && whole < b.end && whole < 16u * kG * kT, f + whole, zero);"):
    assert a in t, a
    t = t.replace(a, a.replace("load16(", "load16nt("), 1)
out = t
