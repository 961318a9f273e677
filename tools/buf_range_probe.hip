// Probe (GPU box): does a raw buffer load's range check include soffset?  A 256-float buffer
// holding 1..256 behind a descriptor of 64 bytes (16 records); loads of one dword and of a dwordx4
// at (voffset, soffset) pairs on both sides of the range.  Prints what each load returned.
//   hipcc --offload-arch=gfx950 -O2 tools/buf_range_probe.hip -o tools/_buf_range_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(const float* buf, float* out) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(buf), (short)0, 64, 0x00020000);
  if (threadIdx.x != 0) return;
  // dword loads: (voffset, soffset)
  out[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, 60, 0, 0));   // in range
  out[1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, 64, 0, 0));   // voffset past
  out[2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, 0, 64, 0));   // soffset past
  out[3] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, 32, 32, 0));  // sum at the end
  // dwordx4 straddling the end: records 14, 15 in range, 16, 17 past
  typedef float f4 __attribute__((ext_vector_type(4)));
  const f4 a = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, 56, 0, 0));
  const f4 b = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, 0, 56, 0));
  for (int i = 0; i < 4; ++i) {
    out[4 + i] = a[i];
    out[8 + i] = b[i];
  }
  // 4-B aligned (not 16-B aligned) dwordx4 in range
  const f4 c = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, 4, 0, 0));
  for (int i = 0; i < 4; ++i) out[12 + i] = c[i];
}

int main() {
  float h[256];
  for (int i = 0; i < 256; ++i) h[i] = (float)(i + 1);
  float *d, *o;
  hipMalloc(&d, sizeof(h));
  hipMalloc(&o, 16 * sizeof(float));
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  hipMemset(o, 0xff, 16 * sizeof(float));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o);
  float r[16];
  hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
  std::printf("dword (v=60,s=0) %g  (v=64,s=0) %g  (v=0,s=64) %g  (v=32,s=32) %g\n", r[0], r[1], r[2], r[3]);
  std::printf("dwordx4 (v=56,s=0): %g %g %g %g\n", r[4], r[5], r[6], r[7]);
  std::printf("dwordx4 (v=0,s=56): %g %g %g %g\n", r[8], r[9], r[10], r[11]);
  std::printf("dwordx4 (v=4,s=0) unaligned: %g %g %g %g\n", r[12], r[13], r[14], r[15]);
  return 0;
}
