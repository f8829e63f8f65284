# A/B: the NaN test per sorted list, right before that list's sort, so the
# first sorts start while the later lists' loads are still in flight (the
# whole-wave test waited for every load before any compare).  Median paths.
s = open("robust.hip").read()
old = """template <int KP, int RULE>
__device__ __forceinline__ float special_floats(const uint32_t (&v)[KP]) {
  if constexpr (RULE == P2P_RULE_MEDIAN) {
    constexpr int Q = KP / 4;
    fk a[Q], b[Q], c[Q], d[Q];
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      a[j].x = __uint_as_float(v[j]);
      b[j].x = __uint_as_float(v[Q + j]);
      c[j].x = __uint_as_float(v[2 * Q + j]);
      d[j].x = __uint_as_float(v[3 * Q + j]);
    }
    sort_full<Q>(a);
    sort_full<Q>(b);
    sort_full<Q>(c);
    sort_full<Q>(d);
    return four_list_median<Q>(a, b, c, d).x;
  } else {"""
new = """template <int Q>
__device__ __forceinline__ uint64_t sorted_list(const uint32_t* v, fk (&a)[Q]) {
  uint64_t m = 0;
#pragma unroll
  for (int j = 0; j < Q / 2; ++j) m |= unordered_mask(__uint_as_float(v[j]), __uint_as_float(v[j + Q / 2]));
#pragma unroll
  for (int j = 0; j < Q; ++j) a[j].x = __uint_as_float(v[j]);
  sort_full<Q>(a);
  return m;
}

template <int KP, int RULE>
__device__ __forceinline__ float special_floats(const uint32_t (&v)[KP], uint64_t& nan) {
  if constexpr (RULE == P2P_RULE_MEDIAN) {
    constexpr int Q = KP / 4;
    fk a[Q], b[Q], c[Q], d[Q];
    nan = sorted_list<Q>(v, a) | sorted_list<Q>(v + Q, b) | sorted_list<Q>(v + 2 * Q, c) |
          sorted_list<Q>(v + 3 * Q, d);
    return four_list_median<Q>(a, b, c, d).x;
  } else {
    nan = 0;"""
assert old in s
s = s.replace(old, new)
old = """    if (!__builtin_amdgcn_readfirstlane(static_cast<int>(wave_has_nan(v)))) return special_floats<KP, RULE>(v);"""
new = """    uint64_t nan = 0;
    float r = 0.f;
    if constexpr (RULE == P2P_RULE_MEDIAN) {
      r = special_floats<KP, RULE>(v, nan);
      if (!__builtin_amdgcn_readfirstlane(static_cast<int>(nan != 0))) return r;
    } else {
      if (!__builtin_amdgcn_readfirstlane(static_cast<int>(wave_has_nan(v)))) return special_floats<KP, RULE>(v, nan);
    }"""
assert old in s
s = s.replace(old, new)
open("robust.hip", "w").write(s)

s = open("robust_pair.hip").read()
old = """  const bool nan = uniform(wave_has_nan(v));"""
new = """  const bool nan = RULE == P2P_RULE_MEDIAN ? false : uniform(wave_has_nan(v));  // median: per list"""
assert old in s
s = s.replace(old, new)
old = """  T p[Q], q[Q];
#pragma unroll
  for (int j = 0; j < Q; ++j) {
    p[j] = from_bits<T>(v[j]);
    q[j] = from_bits<T>(v[Q + j]);
  }
  sort_full<Q>(p);
  sort_full<Q>(q);"""
new = """  T p[Q], q[Q];
  uint64_t nm = 0;
  if constexpr (FLAGS) {
#pragma unroll
    for (int j = 0; j < Q / 2; ++j) nm |= unordered_mask(__uint_as_float(v[j]), __uint_as_float(v[j + Q / 2]));
  }
#pragma unroll
  for (int j = 0; j < Q; ++j) p[j] = from_bits<T>(v[j]);
  sort_full<Q>(p);
  if constexpr (FLAGS) {
#pragma unroll
    for (int j = 0; j < Q / 2; ++j) nm |= unordered_mask(__uint_as_float(v[Q + j]), __uint_as_float(v[Q + j + Q / 2]));
  }
#pragma unroll
  for (int j = 0; j < Q; ++j) q[j] = from_bits<T>(v[Q + j]);
  sort_full<Q>(q);
  if constexpr (FLAGS) nan = uniform(nm != 0);"""
assert old in s
s = s.replace(old, new)
open("robust_pair.hip", "w").write(s)
