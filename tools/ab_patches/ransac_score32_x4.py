"""A/B edit (tools/ab_build.py KCMC_AB_PATCH): the rigid scorer's fp32 phase A loop
(ransac_common.h score32) with two independent accumulator sets (S, clo, chi for the even
and the odd points, summed at the end) and the next pair of points read from LDS while the
current pair is scored (KCMC_AB_VARIANT=x2p), or four points per iteration with two sets
(x4).  The fp32 sum's order changes; its bracket (s32_bracket) holds for any order."""
import os
import sys

variant = os.environ.get("KCMC_AB_VARIANT", "x2p")
p = os.path.join(sys.argv[1], "ransac_common.h")
s = open(p).read()
a = s.index("__device__ __forceinline__ float score32(")
b = s.index("// [lo, hi] around numpy's S of a trial scored by score32")
body = r'''__device__ __forceinline__ float score32(const float4* __restrict__ pk, int N, const Lin32& L, int& clo, int& chi) {
  float S0 = 0.f, S1 = 0.f;
  int l0 = 0, l1 = 0, h0 = 0, h1 = 0;
  auto one = [&](const float4 p, float& S, int& cl, int& ch) {
    f32x2 e = L.t - f32x2{p.z, p.w};
    e = __builtin_elementwise_fma(L.b, f32x2{p.y, p.y}, e);
    e = __builtin_elementwise_fma(L.a, f32x2{p.x, p.x}, e);
    const float q = __builtin_fmaf(e.x, e.x, e.y * e.y);
    S += q;
    cl += q < L.lo ? 1 : 0;
    ch += q <= L.hi ? 1 : 0;
  };
  int k = 0;
''' + ({"x2p": r'''  if (N >= 2) {
    float4 a = pk[0], b = pk[1];
    for (k = 2; k + 2 <= N; k += 2) {
      const float4 na = pk[k], nb = pk[k + 1];
      one(a, S0, l0, h0);
      one(b, S1, l1, h1);
      a = na;
      b = nb;
    }
    one(a, S0, l0, h0);
    one(b, S1, l1, h1);
  }
''', "x4": r'''  for (; k + 4 <= N; k += 4) {
    const float4 a = pk[k], b = pk[k + 1], c = pk[k + 2], d = pk[k + 3];
    one(a, S0, l0, h0);
    one(b, S1, l1, h1);
    one(c, S0, l0, h0);
    one(d, S1, l1, h1);
  }
  for (; k + 2 <= N; k += 2) {
    one(pk[k], S0, l0, h0);
    one(pk[k + 1], S1, l1, h1);
  }
'''}[variant]) + r'''  if (k < N) one(pk[k], S0, l0, h0);
  clo += l0 + l1;
  chi += h0 + h1;
  return S0 + S1;
}

'''
s = s[:a] + body + s[b:]
open(p, "w").write(s)
