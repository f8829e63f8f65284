# A/B: the trimmed-mean pair kernel at 3 waves per SIMD (<= 168 VGPRs) instead of 2.
s = open("robust_pair.hip").read()
old = "__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void robust_pair_kernel("
assert old in s
s = s.replace(old, "__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(3))) void robust_pair_kernel(")
open("robust_pair.hip", "w").write(s)
