"""A/B edit (tools/ab_build.py KCMC_AB_PATCH): the float matcher's top-8 insertion without
the per-distance wave branch (every distance runs the 9-VALU sorted insertion; no
v_cmp / s_and_saveexec / s_cbranch / exec restore) -- tells whether the tile loop is bound
by VALU issue or by the branch's SALU / latency chain."""
import os
import sys

p = os.path.join(sys.argv[1], "match_f32.hip")
s = open(p).read()
for a in ('  "v_cmp_lt_u32 vcc, %[x], %[k7]\\n\\t"                  \\\n',
          '  "s_and_saveexec_b64 %[sv], vcc\\n\\t"                  \\\n',
          '  "s_cbranch_execz 1f\\n\\t"                             \\\n'):
    assert a in s, a
    s = s.replace(a, "")
a = '  "v_min_u32 %[k0], %[k0], %[x]\\n"                      \\\n  "1:\\n\\t"                                             \\\n  "s_or_b64 exec, exec, %[sv]"\n'
assert a in s
s = s.replace(a, '  "v_min_u32 %[k0], %[k0], %[x]\\n"\n')
s = s.replace('[sv] "=&s"(saved)', '[sv] "=s"(saved)')
open(p, "w").write(s)
