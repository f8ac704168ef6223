// Host-side AddressSanitizer driver for libftmi_asan.so (tests/test_asan_host.py): every
// C entry point's argument validation is exercised with invalid arguments — null pointers,
// bad shapes, misaligned pointers, out-of-range options — and must return its FTMI_E_* code
// without touching memory it does not own.  No GPU: these paths return before any launch.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>

#include "ftmi.h"

static int failures = 0;
#define EXPECT(call, code)                                                              \
  do {                                                                                  \
    const int rc__ = (call);                                                            \
    if (rc__ != (code)) {                                                               \
      std::fprintf(stderr, "FAIL %s:%d: %s -> %d, want %d\n", __FILE__, __LINE__, #call, \
                   rc__, (int)(code));                                                  \
      ++failures;                                                                       \
    }                                                                                   \
  } while (0)

int main() {
  if (std::getenv("FTMI_ASAN_SELFTEST")) {  // proves the instrumentation is live
    volatile int *p = new int[4];
    const int v = p[4];  // heap-buffer-overflow: ASan must abort here
    delete[] p;
    return v;
  }
  alignas(16) static float buf[4096];
  float *a = buf;                                      // 16-B aligned, valid host memory
  float *mis = buf + 1;                                // misaligned by 4 B
  const void *pw[8] = {a, a, a, a, a, a, a, a};       // host pointer arrays (read L entries)
  const float *pb[8] = {a, a, a, a, a, a, a, a};
  ftmi_conv_args ca;
  std::memset(&ca, 0, sizeof(ca));

  EXPECT(ftmi_conv1d(nullptr, nullptr), FTMI_E_ARG);
  EXPECT(ftmi_conv1d(&ca, nullptr), FTMI_E_ARG);
  ca.x = a; ca.w = a; ca.y = a; ca.B = 1; ca.T = 4; ca.Cin = 32; ca.N = 8; ca.k = 1;
  ca.x_stride = 32; ca.y_stride = 8; ca.mma = FTMI_MMA_F16X3;
  EXPECT(ftmi_conv1d(&ca, nullptr), FTMI_E_ARG);       // f16x3 without the split planes
  EXPECT(ftmi_conv_bank_split(nullptr, 0, 1, 1, 16, nullptr, nullptr, 4, 8, nullptr, nullptr,
                              nullptr, 0, 1, nullptr, 0, nullptr, 0, nullptr), FTMI_E_ARG);
  EXPECT(ftmi_conv_bank_split(a, 16, 1, 1, 17, a, a, 4, 8, a, a, a, 32, 2, nullptr, 0, nullptr, 0,
                              nullptr), FTMI_E_SHAPE);
  EXPECT(ftmi_conv_bank_split(a, 16, 1, 1, 16, a, a, 17, 8, a, a, a, 32, 2, nullptr, 0, nullptr, 0,
                              nullptr), FTMI_E_UNSUPPORTED);
  EXPECT(ftmi_conv_bank_split(mis, 16, 1, 1, 16, a, a, 4, 8, a, a, a, 32, 2, nullptr, 0, nullptr, 0,
                              nullptr), FTMI_E_ALIGN);
  EXPECT(ftmi_conv_bank_split(a, 16, 1, 1, 16, a, a, 4, 8, a, a, a, 32, 2, nullptr, 0, nullptr, 8,
                              nullptr), FTMI_E_ARG);  // unknown pool_out flag
  EXPECT(ftmi_conv_bank_split(a, 16, 1, 1, 16, a, a, 4, 8, a, a, a, 32, 2, nullptr, 0, nullptr,
                              FTMI_BANK_Y_SPLIT, nullptr), FTMI_E_UNSUPPORTED);
  ca.x_split = 1; ca.mma = FTMI_MMA_F32;
  EXPECT(ftmi_conv1d(&ca, nullptr), FTMI_E_UNSUPPORTED);  // split rows off the f16x3 path
  ca.x_split = 0; ca.mma = FTMI_MMA_F16X3;
  EXPECT(ftmi_highway(nullptr, 0, 1, 32, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 1, nullptr,
                      nullptr), FTMI_E_ARG);
  EXPECT(ftmi_highway(a, 32, 1, 40, a, a, a, a, buf + 1024, 40, 0, nullptr, nullptr), FTMI_E_SHAPE);
  // fused highway stack: L entries of the host pointer arrays are read, never more
  EXPECT(ftmi_highway_stack(nullptr, 80, 10, 80, 256, a, 0, nullptr, nullptr, nullptr, nullptr,
                            nullptr, 0, nullptr, 0, a, 256, nullptr, nullptr), FTMI_E_ARG);
  EXPECT(ftmi_highway_stack(a, 80, 10, 80, 128, a, 8, pw, pb, pb, nullptr, nullptr, 0, nullptr, 0,
                            buf + 2048, 256, nullptr, nullptr), FTMI_E_SHAPE);
  EXPECT(ftmi_highway_stack(a, 80, 10, 80, 256, a, 9, pw, pb, pb, nullptr, nullptr, 0, nullptr, 0,
                            buf + 2048, 256, nullptr, nullptr), FTMI_E_SHAPE);
  EXPECT(ftmi_highway_stack(a, 80, 10, 80, 256, a, 8, pw, pb, pb, a, nullptr, 500, buf + 2048, 500,
                            nullptr, 0, nullptr, nullptr), FTMI_E_SHAPE);
  EXPECT(ftmi_highway_stack(mis, 80, 10, 80, 256, a, 8, pw, pb, pb, nullptr, nullptr, 0, nullptr, 0,
                            buf + 2048, 256, nullptr, nullptr), FTMI_E_ALIGN);
  EXPECT(ftmi_split_weights_f16(nullptr, 4, 4, nullptr, nullptr), FTMI_E_ARG);
  EXPECT(ftmi_split_weights_f16_frag(a, 20, 4, a, nullptr), FTMI_E_SHAPE);
  EXPECT(ftmi_split_weights(a, 4, 4, mis, nullptr), FTMI_E_ALIGN);
  EXPECT(ftmi_rnn_bidir(0, 1, 1, 64, nullptr, 0, 1, nullptr, nullptr, nullptr, nullptr, nullptr,
                        0.f, nullptr, 0, 2, nullptr, nullptr, nullptr), FTMI_E_ARG);
  EXPECT(ftmi_rnn_bidir(0, 1, 1, 64, a, 192, 1, nullptr, nullptr, a, a, nullptr, 0.f, a, 128, 3,
                        nullptr, a, nullptr), FTMI_E_ARG);
  EXPECT(ftmi_rnn_bidir(0, 1, 1, 64, a, 192, 1, nullptr, nullptr, mis, a, nullptr, 0.f, a, 128, 2,
                        nullptr, a, nullptr), FTMI_E_ALIGN);
  EXPECT(ftmi_attention(nullptr, 0, 1, 1, 1, 64, 0, 64, 128, nullptr, 1.f, nullptr, 0, 2, nullptr,
                        nullptr, 0, nullptr), FTMI_E_ARG);
  EXPECT(ftmi_attention(a, 192, 1, 1, 1, 96, 0, 96, 192, nullptr, 1.f, a, 96, 2, nullptr, nullptr,
                        0, nullptr), FTMI_E_UNSUPPORTED);
  EXPECT(ftmi_attention(a, 384, 1, 4, 2, 64, 0, 128, 256, nullptr, 1.f, a, 128, 2, nullptr, mis,
                        1 << 20, nullptr), FTMI_E_ALIGN);
  EXPECT(ftmi_duration_counts(nullptr, 1, 1, 1, 2.f, nullptr, nullptr, nullptr, nullptr), FTMI_E_ARG);
  EXPECT(ftmi_lr_index(nullptr, 1, 1, 1, nullptr, nullptr), FTMI_E_ARG);
  EXPECT(ftmi_rowdot(nullptr, 0, 1, 4, nullptr, nullptr, 1.f, nullptr, nullptr), FTMI_E_ARG);
  EXPECT(ftmi_embedding(nullptr, 4, nullptr, 135, 256, nullptr, nullptr, nullptr), FTMI_E_ARG);
  // sizes / versions / strings (pure host)
  if (ftmi_abi_version() <= 0) ++failures;
  if (ftmi_rnn_workspace_bytes(64, 512, 1) <= 0 || ftmi_attention_workspace_bytes(2, 100, 2, 64) <= 0)
    ++failures;
  if (std::strlen(ftmi_build_id()) != 64) ++failures;
  for (int code : {0, 1001, 1002, 1003, 1004, 12345})
    if (!ftmi_strerror(code) || !*ftmi_strerror(code)) ++failures;
  std::printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
  return failures ? 1 : 0;
}
