# A/B: the key path inlined into the pair kernels, its loads as asm (so GVN
# cannot merge them with the float path's loads and keep those live), and the
# trimmed kernel at 3 waves per SIMD.
import sys
s = open("robust_pair.hip").read()
def rep(old, new, count=1):
    global s
    assert s.count(old) == count, (old, s.count(old))
    s = s.replace(old, new)
rep("__device__ __attribute__((noinline)) float pair_keys(", "__device__ __forceinline__ float pair_keys(", 2)
rep("""  uint32_t v[kHalf];
  load_half(v, P, c0, lane_off, h);
  if constexpr (RULE == P2P_RULE_MEDIAN)""", """  uint32_t v[kHalf];
#pragma unroll
  for (int j = 0; j < kHalf; ++j) {
    const uint64_t row = reinterpret_cast<uint64_t>(table_at(P, h * kHalf + j) + c0);
    asm volatile("global_load_dword %0, %1, %2" : "=v"(v[j]) : "v"(lane_off), "s"(row) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (RULE == P2P_RULE_MEDIAN)""")
if len(sys.argv) < 2 or sys.argv[1] != "2w":
    rep("__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void robust_pair_kernel(",
        "__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(3))) void robust_pair_kernel(")
open("robust_pair.hip", "w").write(s)
