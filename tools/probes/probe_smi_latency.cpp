// GPU-box probe: latency of the amd-smi calls the SMI source makes per sample, and of
// the sysfs files they read, to decide what bounds the 10 Hz+ sampler.
#include <amd_smi/amdsmi.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

using clk = std::chrono::steady_clock;

template <class F>
void bench(const char* name, F f, int n = 300) {
  std::vector<double> us;
  for (int i = 0; i < n; ++i) {
    auto t0 = clk::now();
    f();
    us.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
  }
  std::sort(us.begin(), us.end());
  std::printf("%-40s p50 %8.1f us  p10 %8.1f  p90 %8.1f\n", name, us[n / 2], us[n / 10], us[9 * n / 10]);
}

int main() {
  if (amdsmi_init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return 1;
  uint32_t ns = 0;
  amdsmi_get_socket_handles(&ns, nullptr);
  std::vector<amdsmi_socket_handle> socks(ns);
  amdsmi_get_socket_handles(&ns, socks.data());
  uint32_t np = 0;
  amdsmi_get_processor_handles(socks[0], &np, nullptr);
  std::vector<amdsmi_processor_handle> ph(np);
  amdsmi_get_processor_handles(socks[0], &np, ph.data());
  auto h = ph[0];
  amdsmi_gpu_metrics_t m;
  amdsmi_vram_usage_t v;
  amdsmi_engine_usage_t e;
  amdsmi_power_info_t p;
  int64_t temp = 0;
  bench("amdsmi_get_gpu_metrics_info", [&] { amdsmi_get_gpu_metrics_info(h, &m); });
  bench("amdsmi_get_gpu_vram_usage", [&] { amdsmi_get_gpu_vram_usage(h, &v); });
  bench("amdsmi_get_gpu_activity", [&] { amdsmi_get_gpu_activity(h, &e); });
  bench("amdsmi_get_power_info", [&] { amdsmi_get_power_info(h, &p); });
  bench("amdsmi_get_temp_metric(hotspot)", [&] {
    amdsmi_get_temp_metric(h, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &temp);
  });
  // sysfs files behind them
  char path[256];
  for (int card = 0; card < 16; ++card) {
    std::snprintf(path, sizeof path, "/sys/class/drm/card%d/device/gpu_metrics", card);
    std::ifstream f(path, std::ios::binary);
    if (!f) continue;
    std::string p1 = path;
    bench(("read " + p1).c_str(), [&] {
      std::ifstream g(p1, std::ios::binary);
      char buf[4096];
      g.read(buf, sizeof buf);
    });
    std::snprintf(path, sizeof path, "/sys/class/drm/card%d/device/mem_info_vram_used", card);
    std::string p2 = path;
    bench(("read " + p2).c_str(), [&] {
      std::ifstream g(p2);
      std::string s;
      g >> s;
    });
    break;
  }
  amdsmi_shut_down();
  return 0;
}
