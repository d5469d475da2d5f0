// Host-link copy probe: H2D and D2H alone and at the same time, through the HIP streams, the
// runtime's default SDMA pick (hsa_amd_memory_async_copy) and explicitly chosen SDMA engines
// (hsa_amd_memory_async_copy_on_engine), plus a CU copy kernel over mapped pinned memory.
// Prints one JSON line. Build: hipcc --offload-arch=gfx950 -O2 tools/copy_probe.hip -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

__global__ void k_copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t find_agents(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
  if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
  return HSA_STATUS_SUCCESS;
}
static bool owner(const void* p, hsa_agent_t& a) {
  hsa_amd_pointer_info_t info;
  std::memset(&info, 0, sizeof info);
  info.size = sizeof info;
  if (hsa_amd_pointer_info(p, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return false;
  a = info.agentOwner;
  return info.type != HSA_EXT_POINTER_TYPE_UNKNOWN;
}

int main(int argc, char** argv) {
  const size_t N = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024) << 20;
  const int reps = 3;
  CK(hipSetDevice(0));
  void *h_in, *h_out, *d_in, *d_out;
  CK(hipHostMalloc(&h_in, N, hipHostMallocDefault));
  CK(hipHostMalloc(&h_out, N, hipHostMallocDefault));
  CK(hipMalloc(&d_in, N));
  CK(hipMalloc(&d_out, N));
  std::memset(h_in, 1, N);
  std::memset(h_out, 2, N);
  CK(hipMemset(d_in, 3, N));
  CK(hipMemset(d_out, 4, N));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hsa_iterate_agents(find_agents, nullptr);
  hsa_agent_t gpu, host;
  if (!owner(d_in, gpu) || !owner(h_in, host)) { std::fprintf(stderr, "pointer info failed\n"); return 1; }
  uint32_t st_h2d = 0, st_d2h = 0, pf_h2d = 0, pf_d2h = 0;
  hsa_amd_memory_copy_engine_status(gpu, host, &st_h2d);
  hsa_amd_memory_copy_engine_status(host, gpu, &st_d2h);
  hsa_amd_memory_get_preferred_copy_engine(gpu, host, &pf_h2d);
  hsa_amd_memory_get_preferred_copy_engine(host, gpu, &pf_d2h);
  hsa_signal_t sig;
  hsa_signal_create(0, 0, nullptr, &sig);
  void *m_in = nullptr, *m_out = nullptr;
  CK(hipHostGetDevicePointer(&m_in, h_in, 0));
  CK(hipHostGetDevicePointer(&m_out, h_out, 0));

  auto gbps = [&](double t, int dirs) { return dirs * (double)N / t / 1e9; };
  auto best = [&](auto f) { double b = 1e30; f(); for (int r = 0; r < reps; r++) { double t0 = now(); f(); b = std::min(b, now() - t0); } return b; };
  std::string out = "{";
  char buf[256];
  auto add = [&](const std::string& k, double v) {
    char t[256];
    std::snprintf(t, sizeof t, "%s\"%s\": %.2f", out.size() > 1 ? ", " : "", k.c_str(), v);
    out += t;
  };

  add("h2d_hip", gbps(best([&] { CK(hipMemcpyAsync(d_in, h_in, N, hipMemcpyHostToDevice, s1)); CK(hipStreamSynchronize(s1)); }), 1));
  add("d2h_hip", gbps(best([&] { CK(hipMemcpyAsync(h_out, d_out, N, hipMemcpyDeviceToHost, s2)); CK(hipStreamSynchronize(s2)); }), 1));
  add("both_hip_2streams", gbps(best([&] {
        CK(hipMemcpyAsync(d_in, h_in, N, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(h_out, d_out, N, hipMemcpyDeviceToHost, s2));
        CK(hipStreamSynchronize(s1)); CK(hipStreamSynchronize(s2)); }), 2));
  auto hsa_wait = [&] { hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_BLOCKED); };
  add("both_hsa_default", gbps(best([&] {
        hsa_signal_store_screlease(sig, 2);
        hsa_amd_memory_async_copy(d_in, gpu, h_in, host, N, 0, nullptr, sig);
        hsa_amd_memory_async_copy(h_out, host, d_out, gpu, N, 0, nullptr, sig);
        hsa_wait(); }), 2));
  add("both_hipH2D_hsaD2H", gbps(best([&] {
        hsa_signal_store_screlease(sig, 1);
        CK(hipMemcpyAsync(d_in, h_in, N, hipMemcpyHostToDevice, s1));
        hsa_amd_memory_async_copy(h_out, host, d_out, gpu, N, 0, nullptr, sig);
        CK(hipStreamSynchronize(s1)); hsa_wait(); }), 2));
  // explicit engines: for every pair (a for H2D, b for D2H) of the first 4 engines the status reports
  std::vector<int> eng;
  for (int e = 0; e < 16 && eng.size() < 4; e++) if ((st_h2d | st_d2h) >> e & 1) eng.push_back(e);
  double best_pair = 0; int ba = -1, bb = -1;
  for (int a : eng) {
    hsa_signal_store_screlease(sig, 1);
    double t0 = now();
    hsa_status_t r = hsa_amd_memory_async_copy_on_engine(d_in, gpu, h_in, host, N, 0, nullptr, sig, (hsa_amd_sdma_engine_id_t)(1u << a), true);
    if (r != HSA_STATUS_SUCCESS) { hsa_signal_store_screlease(sig, 0); continue; }
    hsa_wait();
    add("h2d_engine" + std::to_string(a), gbps(now() - t0, 1));
    hsa_signal_store_screlease(sig, 1);
    t0 = now();
    r = hsa_amd_memory_async_copy_on_engine(h_out, host, d_out, gpu, N, 0, nullptr, sig, (hsa_amd_sdma_engine_id_t)(1u << a), true);
    if (r != HSA_STATUS_SUCCESS) { hsa_signal_store_screlease(sig, 0); continue; }
    hsa_wait();
    add("d2h_engine" + std::to_string(a), gbps(now() - t0, 1));
  }
  for (int a : eng) for (int b : eng) {
    if (a == b) continue;
    double t = best([&] {
      hsa_signal_store_screlease(sig, 2);
      if (hsa_amd_memory_async_copy_on_engine(d_in, gpu, h_in, host, N, 0, nullptr, sig, (hsa_amd_sdma_engine_id_t)(1u << a), true) != HSA_STATUS_SUCCESS) hsa_signal_subtract_screlease(sig, 1);
      if (hsa_amd_memory_async_copy_on_engine(h_out, host, d_out, gpu, N, 0, nullptr, sig, (hsa_amd_sdma_engine_id_t)(1u << b), true) != HSA_STATUS_SUCCESS) hsa_signal_subtract_screlease(sig, 1);
      hsa_wait(); });
    add("both_engines_" + std::to_string(a) + "_" + std::to_string(b), gbps(t, 2));
    if (gbps(t, 2) > best_pair) { best_pair = gbps(t, 2); ba = a; bb = b; }
  }
  // CU copy kernels over mapped pinned memory
  add("d2h_kernel", gbps(best([&] { k_copy16<<<1024, 256, 0, s2>>>((const uint4*)d_out, (uint4*)m_out, N / 16); CK(hipStreamSynchronize(s2)); }), 1));
  add("h2d_kernel", gbps(best([&] { k_copy16<<<1024, 256, 0, s1>>>((const uint4*)m_in, (uint4*)d_in, N / 16); CK(hipStreamSynchronize(s1)); }), 1));
  add("both_hipH2D_kernelD2H", gbps(best([&] {
        CK(hipMemcpyAsync(d_in, h_in, N, hipMemcpyHostToDevice, s1));
        k_copy16<<<1024, 256, 0, s2>>>((const uint4*)d_out, (uint4*)m_out, N / 16);
        CK(hipStreamSynchronize(s1)); CK(hipStreamSynchronize(s2)); }), 2));
  add("both_kernels", gbps(best([&] {
        k_copy16<<<512, 256, 0, s1>>>((const uint4*)m_in, (uint4*)d_in, N / 16);
        k_copy16<<<512, 256, 0, s2>>>((const uint4*)d_out, (uint4*)m_out, N / 16);
        CK(hipStreamSynchronize(s1)); CK(hipStreamSynchronize(s2)); }), 2));
  std::snprintf(buf, sizeof buf, ", \"mb\": %zu, \"status_h2d\": %u, \"status_d2h\": %u, \"preferred_h2d\": %u, \"preferred_d2h\": %u, \"best_pair\": [%d, %d]}",
                N >> 20, st_h2d, st_d2h, pf_h2d, pf_d2h, ba, bb);
  out += buf;
  std::printf("%s\n", out.c_str());
  return 0;
}
