# A/B: the parity-merge trimmed kernel at 3 waves per SIMD: the parity hand-off
# runs through ONE 16 KB region in sequence (wave 0 -> wave 1, then wave 1 ->
# wave 0, one more barrier), so a block needs 26.9 KB of LDS (6 blocks per CU)
# and the kernel asks for 3 waves per SIMD (168 VGPRs).
s = open("robust_pair.hip").read()
def rep(old, new):
    global s
    assert s.count(old) == 1, old[:80]
    s = s.replace(old, new)
rep('''  Img r0 = im, r1 = im + kHalf / 8 * 64;
  if (h == 0) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int g = 0; g < kHalf / 8; ++g)
      r0[g * 64 + lane] = u32x4{raw(x[8 * g + 1]), raw(x[8 * g + 3]), raw(x[8 * g + 5]), raw(x[8 * g + 7])};
  } else {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int g = 0; g < kHalf / 8; ++g)
      r1[g * 64 + lane] = u32x4{raw(x[8 * g]), raw(x[8 * g + 2]), raw(x[8 * g + 4]), raw(x[8 * g + 6])};
  }''', '''  Img r0 = im, r1 = im + kHalf / 8 * 64;  // r0: the one hand-off region; r1: wave 1's crossing values
  if (h == 0) {
#pragma unroll
    for (int g = 0; g < kHalf / 8; ++g)
      r0[g * 64 + lane] = u32x4{raw(x[8 * g + 1]), raw(x[8 * g + 3]), raw(x[8 * g + 5]), raw(x[8 * g + 7])};
  }''')
rep('''    auto part = (float __attribute__((address_space(3)))*)(im + kHalf / 4 * 64);''',
    '''    auto part = (float __attribute__((address_space(3)))*)(im + (kHalf / 8 + 10) * 64);''')
rep('''    T m[kHalf];
    if (h == 0) {  // v = merge(A_even, B_even): ranks I0..I1 of it
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        m[j] = x[2 * j];
        m[Q + j] = from_raw<T>(img_at(r1, j, lane));
      }
      net_merge128_r26_102<true>(m);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      send_run<I0, NX>(r1, m, lane);
    } else {       // w = merge(A_odd, B_odd): ranks I0-1..I1-1
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        m[j] = from_raw<T>(img_at(r0, j, lane));
        m[Q + j] = x[2 * j + 1];
      }
      net_merge128_r25_101<true>(m);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      send_run<IM - 1, NX>(r0, m, lane);
    }''', '''    T m[kHalf];
    if (h == 1) {  // A_odd out of r0, then B_even into it
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        m[j] = from_raw<T>(img_at(r0, j, lane));
        m[Q + j] = x[2 * j + 1];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int g = 0; g < kHalf / 8; ++g)
        r0[g * 64 + lane] = u32x4{raw(x[8 * g]), raw(x[8 * g + 2]), raw(x[8 * g + 4]), raw(x[8 * g + 6])};
    }
    block_sync();  // 1b: B_even in r0
    if (h == 0) {  // v = merge(A_even, B_even): ranks I0..I1 of it
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        m[j] = x[2 * j];
        m[Q + j] = from_raw<T>(img_at(r0, j, lane));
      }
      net_merge128_r26_102<true>(m);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      send_run<I0, NX>(r0, m, lane);
    } else {       // w = merge(A_odd, B_odd): ranks I0-1..I1-1
      net_merge128_r25_101<true>(m);
      send_run<IM - 1, NX>(r1, m, lane);
    }''')
rep('''        const T vi = from_raw<T>(img_at(r1, i - I0, lane));''', '''        const T vi = from_raw<T>(img_at(r0, i - I0, lane));''')
rep('''      c[2 * (IM - I0)] = min(from_raw<T>(img_at(r1, IM - I0, lane)), m[IM - 1]);''', '''      c[2 * (IM - I0)] = min(from_raw<T>(img_at(r0, IM - I0, lane)), m[IM - 1]);''')
rep('''    c[0] = max(m[IM], from_raw<T>(img_at(r0, 0, lane)));''', '''    c[0] = max(m[IM], from_raw<T>(img_at(r1, 0, lane)));''')
rep('''      const T wi = from_raw<T>(img_at(r0, i - IM, lane));  // w_{i-1}''', '''      const T wi = from_raw<T>(img_at(r1, i - IM, lane));  // w_{i-1}''')
rep("__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void robust_pair_kernel(",
    "__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(3))) void robust_pair_kernel(")
rep("  __shared__ u32x4 img_raw[kHalf / 4 * 64 + 16];", "  __shared__ u32x4 img_raw[(kHalf / 8 + 10) * 64 + 16];")
open("robust_pair.hip", "w").write(s)
