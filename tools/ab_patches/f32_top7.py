"""A/B edit (tools/ab_build.py KCMC_AB_PATCH): the float matcher's per-lane list at 7 keys
instead of 8 (one v_med3 fewer per insertion and a lower insertion rate, more rows for the
exact fallback)."""
import os
import sys

p = os.path.join(sys.argv[1], "match_f32.hip")
s = open(p).read()
for a, b in (("constexpr int kTop = 8;", "constexpr int kTop = 7;"),
             ('static_assert(kTop == 8, "topk_try keeps a top-8");', 'static_assert(kTop == 7, "top-7 variant");'),
             ('"v_cmp_lt_u32 vcc, %[x], %[k7]\\n\\t"', '"v_cmp_lt_u32 vcc, %[x], %[k6]\\n\\t"'),
             ('  "v_med3_u32 %[k7], %[k6], %[k7], %[x]\\n\\t"           \\\n', ''),
             ('[k6] "+v"(k[6]), [k7] "+v"(k[7]),', '[k6] "+v"(k[6]),')):
    assert a in s, a
    s = s.replace(a, b)
open(p, "w").write(s)
