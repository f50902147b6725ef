"""A/B edit (tools/ab_build.py KCMC_AB_PATCH): the float matcher's insertion threshold shared by
the two lane halves of a template row: at every tile, th = min(own 8th key, partner's 8th key)
(lane ^ 32 holds the same template row's other frame rows).  A value >= the partner's 8th key
cannot be among the row's 8 best (the partner already holds 8 smaller ones), so rejecting it
keeps the certification bound (the merged list's 8th value); fewer values insert."""
import os
import sys

p = os.path.join(sys.argv[1], "match_f32.hip")
s = open(p).read()
rep = [
    ('"v_cmp_lt_u32 vcc, %[x], %[k7]\\n\\t"', '"v_cmp_lt_u32 vcc, %[x], %[th]\\n\\t"'),
    ('  "v_min_u32 %[k0], %[k0], %[x]\\n"                      \\\n',
     '  "v_min_u32 %[k0], %[k0], %[x]\\n\\t"                    \\\n  "v_min_u32 %[th], %[th], %[k7]\\n"                    \\\n'),
    ('[x] "+v"(xb), [sv] "=&s"(saved)', '[x] "+v"(xb), [th] "+v"(th), [sv] "=&s"(saved)'),
    ('__device__ __forceinline__ void topk_try(uint32_t (&k)[kTop], uint32_t xb, uint32_t kmask, uint32_t id) {',
     '__device__ __forceinline__ void topk_try(uint32_t (&k)[kTop], uint32_t xb, uint32_t kmask, uint32_t id, uint32_t& th) {'),
    ('        topk_try<true>(ck[b], __float_as_uint(acc[b][0]), kmask, (uint32_t)(hh * 16) | tbase);',
     '        topk_try<true>(ck[b], __float_as_uint(acc[b][0]), kmask, (uint32_t)(hh * 16) | tbase, th[b]);'),
    ('          topk_try<false>(ck[b], __float_as_uint(acc[b][r]), kmask, (uint32_t)(hh * 16 + r) | tbase);',
     '          topk_try<false>(ck[b], __float_as_uint(acc[b][r]), kmask, (uint32_t)(hh * 16 + r) | tbase, th[b]);'),
    ('    const uint32_t tbase = (uint32_t)t << 5;',
     '    const uint32_t tbase = (uint32_t)t << 5;\n    uint32_t th[kBlk];\n#pragma unroll\n    for (int b = 0; b < kBlk; ++b)\n'
     '      th[b] = min(ck[b][kTop - 1], (uint32_t)__shfl_xor((int)ck[b][kTop - 1], 32));'),
]
for a, b in rep:
    assert a in s, a
    s = s.replace(a, b)
open(p, "w").write(s)
