# A/B: the median pair kernel's first two-set level split between the waves:
# each wave half-cleans its own kept set and they swap its max (one more
# barrier), so wave 1 hands over 32 keys (8 KB) instead of 64 and wave 0's
# tail (run while wave 1 has exited) shrinks by about a quarter.
s = open("robust_pair.hip").read()
old = """  if (h == 1) {
#pragma unroll
    for (int g = 0; g < Q / 4; ++g) im[g * 64 + lane] = u32x4{raw(x[4 * g]), raw(x[4 * g + 1]), raw(x[4 * g + 2]), raw(x[4 * g + 3])};
  }
  block_sync();  // 2: B's kept half in the image
  if (h == 1) return 0.f;
  T y[Q];
#pragma unroll
  for (int j = 0; j < Q; ++j) y[j] = from_raw<T>(img_at(im, j, lane));
  return val(two_set_median<Q>(x, y));
}"""
new = """  // first level of the two-set search, each wave on its own kept set
  constexpr int H = Q / 2;
  T xl[H];
#pragma unroll
  for (int i = 0; i < H; ++i) xl[i] = min(x[i], x[i + H]);
  const T mx = max_tree<H>(xl);
  auto part2 = (uint32_t __attribute__((address_space(3)))*)(im + H / 4 * 64);  // past the 8 KB hand-off
  part2[h * 64 + lane] = raw(mx);
  block_sync();  // 2: both max(lo) of the kept sets
  const T mo2 = from_raw<T>(part2[(1 - h) * 64 + lane]);
  const bool d2 = h == 0 ? le(mx, mo2) : le(mo2, mx);  // max(X_lo) <= max(Y_lo): X_hi u Y_lo
  const T lim2 = keep_limit(T{}, d2 == (h == 0));
  T x2[H];
#pragma unroll
  for (int i = 0; i < H; ++i) x2[i] = keep(x[i], x[i + H], lim2);
  if (h == 1) {
#pragma unroll
    for (int g = 0; g < H / 4; ++g) im[g * 64 + lane] = u32x4{raw(x2[4 * g]), raw(x2[4 * g + 1]), raw(x2[4 * g + 2]), raw(x2[4 * g + 3])};
  }
  block_sync();  // 3: B's kept quarter in the image
  if (h == 1) return 0.f;
  T y2[H];
#pragma unroll
  for (int j = 0; j < H; ++j) y2[j] = from_raw<T>(img_at(im, j, lane));
  return val(two_set_median<H>(x2, y2));
}"""
assert s.count(old) == 1
s = s.replace(old, new)
open("robust_pair.hip", "w").write(s)
