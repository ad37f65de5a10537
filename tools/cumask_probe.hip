// Where do the workgroups of a CU-masked stream (hipExtStreamCreateWithCUMask) run on MI355X? One probe kernel records
// each workgroup's XCC / SE / SH / CU from the hardware-id registers (scalar register READS only); printed per mask:
// the distinct CUs used per XCD. Masks tried: all bits, the low half of the bits, every 8th bit cleared, and
// bits [k*32, k*32+4) cleared for every 32-bit word (4 of every 32). Used to size a stream that leaves a few CUs of
// every XCD to a concurrent memory-bound kernel.
//   hipcc --offload-arch=gfx950 -O3 tools/cumask_probe.hip -o /tmp/cumask_probe && /tmp/cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdint>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void ids(uint32_t* out) {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
  // keep the workgroup resident a little, so the dispatcher spreads the grid over every CU it may use
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < 20000) {
  }
}

static void report(const char* name, hipStream_t s, uint32_t* d, int blocks) {
  ids<<<blocks, 64, 0, s>>>(d);
  if (hipStreamSynchronize(s) != hipSuccess) { printf("%s: sync failed\n", name); return; }
  std::vector<uint32_t> h(2 * blocks);
  (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  std::set<std::tuple<int, int, int, int>> cus;
  for (int b = 0; b < blocks; ++b) {
    const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
    const int cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
    cus.insert({(int)xcc, se, sh, cu});
  }
  int per[16] = {0};
  for (auto& c : cus) per[std::get<0>(c)]++;
  printf("%-34s %4zu CUs:", name, cus.size());
  for (int x = 0; x < 8; ++x) printf(" xcd%d=%d", x, per[x]);
  printf("\n");
}

int main() {
  int dev = 0, ncu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  printf("CUs: %d\n", ncu);
  uint32_t* d;
  const int blocks = 4096;
  (void)hipMalloc(&d, 2 * blocks * 4);
  report("default stream", 0, d, blocks);
  const int words = (ncu + 31) / 32;
  struct M { const char* name; std::vector<uint32_t> m; };
  std::vector<M> masks;
  masks.push_back({"all bits", std::vector<uint32_t>(words, 0xffffffffu)});
  {
    std::vector<uint32_t> m(words, 0);
    for (int i = 0; i < ncu / 2; ++i) m[i / 32] |= 1u << (i % 32);
    masks.push_back({"bits [0, ncu/2)", m});
  }
  {
    std::vector<uint32_t> m(words, 0xffffffffu);
    for (int i = 0; i < ncu; i += 8) m[i / 32] &= ~(1u << (i % 32));
    masks.push_back({"every 8th bit cleared", m});
  }
  {
    std::vector<uint32_t> m(words, 0xffffffffu);
    for (int w = 0; w < words; ++w) m[w] &= ~0xfu;
    masks.push_back({"4 of every 32 bits cleared", m});
  }
  {
    std::vector<uint32_t> m(words, 0);
    for (int i = 0; i < ncu; i += 8) m[i / 32] |= 1u << (i % 32);
    masks.push_back({"every 8th bit only", m});
  }
  for (auto& mk : masks) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mk.m.size(), mk.m.data()) != hipSuccess) {
      printf("%s: hipExtStreamCreateWithCUMask failed\n", mk.name);
      continue;
    }
    report(mk.name, s, d, blocks);
    (void)hipStreamDestroy(s);
  }
  return 0;
}
