// Accuracy of the hardware reciprocal seeds on gfx950 (v_rcp_f64, v_rcp_f32 of a double
// rounded to float) against the IEEE quotient 1/q, q = 1 + e^t over t in [-40, 80]: max
// relative error of the seed, after one and after two Newton steps.  Used to size the Newton
// chain of k_logistic_coef (csrc/complete_grad.hip).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

__global__ void k(int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double t = -40.0 + 120.0 * (double)i / (double)n;
  const double q = 1.0 + exp(t);
  const double ref = 1.0 / q;
  double y64 = __builtin_amdgcn_rcp(q);
  double y32 = (double)__builtin_amdgcn_rcpf((float)q);
  double r[6];
  r[0] = fabs(y64 - ref) / ref;
  r[1] = fabs(y32 - ref) / ref;
  y64 = __builtin_fma(__builtin_fma(-q, y64, 1.0), y64, y64);
  y32 = __builtin_fma(__builtin_fma(-q, y32, 1.0), y32, y32);
  r[2] = fabs(y64 - ref) / ref;
  r[3] = fabs(y32 - ref) / ref;
  y64 = __builtin_fma(__builtin_fma(-q, y64, 1.0), y64, y64);
  y32 = __builtin_fma(__builtin_fma(-q, y32, 1.0), y32, y32);
  r[4] = fabs(y64 - ref) / ref;
  r[5] = fabs(y32 - ref) / ref;
  for (int c = 0; c < 6; ++c) out[(size_t)c * n + i] = r[c];
}

int main() {
  const int n = 1 << 22;
  double* d;
  if (hipMalloc(&d, sizeof(double) * 6 * n) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, n, d);
  static double h[6 * (1 << 22)];
  if (hipMemcpy(h, d, sizeof(double) * 6 * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  const char* names[6] = {"rcp_f64 seed", "rcp_f32 seed", "rcp_f64 + 1 Newton",
                          "rcp_f32 + 1 Newton", "rcp_f64 + 2 Newton", "rcp_f32 + 2 Newton"};
  for (int c = 0; c < 6; ++c) {
    double m = 0;
    for (int i = 0; i < n; ++i) m = fmax(m, h[(size_t)c * n + i]);
    printf("%-20s max rel err %.3e (%.1f ulp)\n", names[c], m, m / 2.220446049250313e-16);
  }
  (void)hipFree(d);
  return 0;
}
