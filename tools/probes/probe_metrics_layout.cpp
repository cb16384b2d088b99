// GPU-box probe: where do the interconnect fields of the SMU metrics table sit in the
// raw sysfs blob? Prints, for GPU 0, the raw `gpu_metrics` blob read just before and
// just after one amdsmi_get_gpu_metrics_info() call (hex, 8 B words) and the values
// amd-smi decoded for the accumulator / bandwidth / per-XCC fields, so the offsets can
// be read off and hard-coded next to kFormat1Layout (csrc/sources.cpp) - where they are
// verified against amd-smi again at every start-up.
//
//   hipcc -O2 probe_metrics_layout.cpp -lamd_smi
#include <amd_smi/amdsmi.h>
#include <fcntl.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <vector>

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
  uint64_t bdf = 0;
  amdsmi_get_gpu_bdf_id(h, &bdf);
  char path[160];
  std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%04x:%02x:%02x.%x/gpu_metrics", unsigned(bdf >> 32),
                unsigned((bdf >> 8) & 0xFF), unsigned((bdf >> 3) & 0x1F), unsigned(bdf & 0x7));
  const int fd = ::open(path, O_RDONLY);
  if (fd < 0) return 2;
  std::vector<uint8_t> a(8192), b(8192);
  amdsmi_gpu_metrics_t m{};
  const ssize_t na = ::pread(fd, a.data(), a.size(), 0);
  amdsmi_get_gpu_metrics_info(h, &m);
  const ssize_t nb = ::pread(fd, b.data(), b.size(), 0);
  std::printf("path %s sizes %zd %zd\n", path, na, nb);
  auto u64 = [](unsigned long long x) { return x; };
  std::printf("energy_accumulator %llu\n", u64(m.energy_accumulator));
  std::printf("system_clock_counter %llu\n", u64(m.system_clock_counter));
  std::printf("firmware_timestamp %llu\n", u64(m.firmware_timestamp));
  std::printf("pcie_bandwidth_acc %llu\n", u64(m.pcie_bandwidth_acc));
  std::printf("pcie_bandwidth_inst %llu\n", u64(m.pcie_bandwidth_inst));
  std::printf("pcie_link_width %u pcie_link_speed %u\n", m.pcie_link_width, m.pcie_link_speed);
  std::printf("xgmi_link_width %u xgmi_link_speed %u\n", m.xgmi_link_width, m.xgmi_link_speed);
  std::printf("gfx_activity_acc %u mem_activity_acc %u\n", m.gfx_activity_acc, m.mem_activity_acc);
  std::printf("num_partition %u current_uclk %u\n", m.num_partition, m.current_uclk);
  for (int i = 0; i < AMDSMI_MAX_NUM_XGMI_LINKS; ++i)
    std::printf("xgmi[%d] read_acc %llu write_acc %llu status %u\n", i, u64(m.xgmi_read_data_acc[i]),
                u64(m.xgmi_write_data_acc[i]), m.xgmi_link_status[i]);
  for (int i = 0; i < AMDSMI_MAX_NUM_XCC; ++i)
    std::printf("xcp0 gfx_busy_inst[%d] %u gfx_busy_acc %llu\n", i, m.xcp_stats[0].gfx_busy_inst[i],
                u64(m.xcp_stats[0].gfx_busy_acc[i]));
  for (int i = 0; i < AMDSMI_MAX_NUM_GFX_CLKS; ++i) std::printf("current_gfxclks[%d] %u\n", i, m.current_gfxclks[i]);
  for (int k = 0; k < 2; ++k) {
    const auto& v = k ? b : a;
    const ssize_t n = k ? nb : na;
    std::printf("raw%c", k ? 'B' : 'A');
    for (ssize_t off = 0; off + 8 <= n; off += 8) {
      unsigned long long w = 0;
      for (int j = 0; j < 8; ++j) w |= (unsigned long long)v[off + j] << (8 * j);
      std::printf(" %zd:%llx", off, w);
    }
    std::printf("\n");
  }
  ::close(fd);
  amdsmi_shut_down();
  return 0;
}
