# A/B: wave 1 also half-cleans its kept half (level 1 of the search) and
# hands over Y_lo / Y_hi + max(Y_lo); wave 0 reads only the half it keeps.
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
  return val(two_set_median<Q>(x, y));"""
new = """  constexpr int H = Q / 2;
  if (h == 1) {  // Y_lo in slots 0..7, Y_hi in slots 8..15, max(Y_lo) in part[128 + lane]
    T yl[H];
#pragma unroll
    for (int i = 0; i < H; ++i) yl[i] = min(x[i], x[i + H]);
#pragma unroll
    for (int g = 0; g < H / 4; ++g) im[g * 64 + lane] = u32x4{raw(yl[4 * g]), raw(yl[4 * g + 1]), raw(yl[4 * g + 2]), raw(yl[4 * g + 3])};
#pragma unroll
    for (int g = 0; g < H / 4; ++g) {
      u32x4 u;
#pragma unroll
      for (int k = 0; k < 4; ++k) u[k] = raw(max(x[4 * g + k], x[4 * g + k + H]));
      im[(H / 4 + g) * 64 + lane] = u;
    }
    part[128 + lane] = raw(max_tree<H>(yl));
  }
  block_sync();  // 2: B's kept half, half-cleaned, in the image
  if (h == 1) return 0.f;
  T xl[H];
#pragma unroll
  for (int i = 0; i < H; ++i) xl[i] = min(x[i], x[i + H]);
  const bool d1 = le(max_tree<H>(xl), from_raw<T>(part[128 + lane]));  // keep X_hi, Y_lo
  const Img yb = im + (d1 ? 0 : H / 4 * 64);
  const T l1 = keep_limit(T{}, d1);
  T x2[H], y2[H];
#pragma unroll
  for (int i = 0; i < H; ++i) y2[i] = from_raw<T>(img_at(yb, i, lane));
#pragma unroll
  for (int i = 0; i < H; ++i) x2[i] = keep(x[i], x[i + H], l1);
  return val(two_set_median<H>(x2, y2));"""
assert old in s
s = s.replace(old, new)
old = "  __shared__ u32x4 img_raw[kHalf / 8 * 64 + 32];"
assert old in s
s = s.replace(old, "  __shared__ u32x4 img_raw[kHalf / 8 * 64 + 48];")
open("robust_pair.hip", "w").write(s)
