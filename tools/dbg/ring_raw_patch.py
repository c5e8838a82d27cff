# Build-variant edit: the ring kernel's consumers release a chunk as soon as
# it is published and do nothing else (timing of the loader's stream alone;
# records are not written)
t = s
a = "    const uint32_t chunk = c0 + t;\n    const uint32_t pos = q->pos[e], npc = q->npc[e], span = q->span[e];"
assert a in t
t = t.replace(a, "    if (lane == 0) lds_store(&q->done[e], t + 1u);\n    continue;\n" + a, 1)
out = t
