set -e
cd /root/repo
B=tools/build_variant.sh
bash $B abl_v6hash 's.replace("""    for (int k = 12; k < 36; k++) {
      const uint32_t b = byte_at(d, k < 32 ? 22 + k : 54 + (k - 32));
      h ^= T6[((k - 12) << 8) | b];
    }""", "")' | tail -1
bash $B abl_v4hash 's.replace("""    for (int k = 0; k < 4; k++) {
      hx ^= T.look(k, (sb >> (8 * k)) & 0xffu);
      hx ^= T.look(4 + k, (db >> (8 * k)) & 0xffu);
      hx ^= T.look(8 + k, (pb >> (8 * k)) & 0xffu);
    }""", "    hx = ((uint64_t)(sb ^ pb) << 32) | (db ^ sb);")' | tail -1
bash $B abl_csum 's.replace("for (int k = 4; k < kPrefixDw; k++) C[k + 1] = add1c(C[k], d[k]);", "for (int k = 4; k < kPrefixDw; k++) C[k + 1] = d[k];")' | tail -1
bash $B abl_mux 's.replace("window<4>(src4, qs, h);", "h[0] = src4[0]; h[1] = src4[1]; h[2] = src4[2]; h[3] = src4[3];").replace("spre = add1c(select<4>(Cq, qs), h0 & 0xffffu);", "spre = add1c(Cq[0], h0 & 0xffffu);").replace("const uint32_t s_e = add1c(select<4>(Ce, qi), select<4>(de, qi) & ones(e & 3));", "const uint32_t s_e = add1c(Ce[0], de[0] & ones(e & 3));")' | tail -1
python3 - <<'PY'
import re
s=open('/root/repo/ix_amd/csrc/ixgrx_kernels.hip').read()
i=s.index('  uint32_t flags = s.flags;\n  if (s.l4_kind == 1)')
j=s.index('  Rec r;\n  r.w0 = (s.fg & 0xffffu)')
body=s[i:j]
open('/tmp/rec_body.txt','w').write(body)
PY
bash $B abl_rec 's.replace(open("/tmp/rec_body.txt").read(), "  uint32_t flags = s.flags | (l4_res << 8), v = s.proto ^ etype ^ ver ^ ihl ^ ip_len ^ (uint32_t)frag, off = s.l4, len = s.l4len, bucket = s.bucket, tfl = s.tcp_flags;\n")' | tail -1
