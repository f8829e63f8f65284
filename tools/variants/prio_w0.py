# A/B: static s_setprio 1 for wave 0 of every median pair block (MI355X guide,
# "Two waves per SIMD" item 4).
s = open("robust_pair.hip").read()
old = """  __shared__ u32x4 img_raw[kHalf / 8 * 64 + 32];
  __shared__ int nan_flag[2];
  const int64_t t = tile_id(gx);"""
assert old in s
s = s.replace(old, old + "\n  if (__builtin_amdgcn_readfirstlane(static_cast<int>(tid_x() >> 6)) == 0) __builtin_amdgcn_s_setprio(1);")
open("robust_pair.hip", "w").write(s)
