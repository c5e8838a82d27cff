# Build-variant edit: the span kernel reads each lane's prefix with six
# ds_read_b128 at the frame's (4-byte aligned) offsets + one ds_read_b32,
# relying on LDS unaligned-access mode, instead of 21 + 4 ds_read_b32.
t = s
a = """#pragma unroll
        for (int k = 3; k < kPrefixDw; k++) d[k] = f[k];
        if (wave_any(L > (uint32_t)kStreamBase)) v96 = u32x4{f[24], f[25], f[26], f[27]};"""
b = """        {
          u32x4 r1, r2, r3, r4, r5, r6;
          uint32_t r0;
          asm volatile("ds_read_b32 %0, %7 offset:12\\n\\t"
                       "ds_read_b128 %1, %7 offset:16\\n\\t"
                       "ds_read_b128 %2, %7 offset:32\\n\\t"
                       "ds_read_b128 %3, %7 offset:48\\n\\t"
                       "ds_read_b128 %4, %7 offset:64\\n\\t"
                       "ds_read_b128 %5, %7 offset:80\\n\\t"
                       "ds_read_b128 %6, %7 offset:96\\n\\t"
                       "s_waitcnt lgkmcnt(0)"
                       : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6)
                       : "v"(f) : "memory");
          d[3] = r0;
          d[4] = r1.x; d[5] = r1.y; d[6] = r1.z; d[7] = r1.w;
          d[8] = r2.x; d[9] = r2.y; d[10] = r2.z; d[11] = r2.w;
          d[12] = r3.x; d[13] = r3.y; d[14] = r3.z; d[15] = r3.w;
          d[16] = r4.x; d[17] = r4.y; d[18] = r4.z; d[19] = r4.w;
          d[20] = r5.x; d[21] = r5.y; d[22] = r5.z; d[23] = r5.w;
          v96 = r6;
        }"""
assert a in t
t = t.replace(a, b, 1)
out = t
