// GPU-box probe: which amd-smi calls work for an unprivileged user on MI355X.
#include <amd_smi/amdsmi.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CHK(x) do { amdsmi_status_t s_ = (x); if (s_ != AMDSMI_STATUS_SUCCESS) { const char* m=nullptr; amdsmi_status_code_to_string(s_, &m); std::printf("  %-40s -> status %d (%s)\n", #x, (int)s_, m?m:"?"); } } while (0)

int main() {
  amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  std::printf("amdsmi_init -> %d\n", (int)st);
  uint32_t ns = 0;
  CHK(amdsmi_get_socket_handles(&ns, nullptr));
  std::vector<amdsmi_socket_handle> socks(ns);
  CHK(amdsmi_get_socket_handles(&ns, socks.data()));
  std::printf("sockets=%u\n", ns);
  for (uint32_t s = 0; s < ns; ++s) {
    uint32_t np = 0;
    CHK(amdsmi_get_processor_handles(socks[s], &np, nullptr));
    std::vector<amdsmi_processor_handle> ph(np);
    CHK(amdsmi_get_processor_handles(socks[s], &np, ph.data()));
    for (uint32_t p = 0; p < np; ++p) {
      auto h = ph[p];
      uint64_t bdf = 0; CHK(amdsmi_get_gpu_bdf_id(h, &bdf));
      amdsmi_board_info_t b{}; CHK(amdsmi_get_gpu_board_info(h, &b));
      amdsmi_asic_info_t a{}; CHK(amdsmi_get_gpu_asic_info(h, &a));
      amdsmi_power_info_t pw{}; CHK(amdsmi_get_power_info(h, &pw));
      amdsmi_vram_usage_t v{}; CHK(amdsmi_get_gpu_vram_usage(h, &v));
      amdsmi_engine_usage_t e{}; CHK(amdsmi_get_gpu_activity(h, &e));
      amdsmi_gpu_metrics_t m{}; CHK(amdsmi_get_gpu_metrics_info(h, &m));
      std::printf("sock %u proc %u bdf=%lx model_number='%s' product='%s' market='%s' \n", s, p, (unsigned long)bdf, b.model_number, b.product_name, a.market_name);
      std::printf("  power: socket=%lu cur=%u avg=%u limit=%u\n", (unsigned long)pw.socket_power, pw.current_socket_power, pw.average_socket_power, pw.power_limit);
      std::printf("  vram total=%u used=%u MB; activity gfx=%u umc=%u mm=%u\n", v.vram_total, v.vram_used, e.gfx_activity, e.umc_activity, e.mm_activity);
      std::printf("  metrics fmt=%u.%u size=%u temp_edge=%u hotspot=%u mem=%u gfx_act=%u umc_act=%u cur_sock_pw=%u avg_sock_pw=%u energy=%lu ts=%lu gfxclk=%u\n",
        m.common_header.format_revision, m.common_header.content_revision, m.common_header.structure_size,
        m.temperature_edge, m.temperature_hotspot, m.temperature_mem, m.average_gfx_activity, m.average_umc_activity,
        m.current_socket_power, m.average_socket_power, (unsigned long)m.energy_accumulator, (unsigned long)m.system_clock_counter, m.current_gfxclk);
      std::printf("  gfx_activity_acc=%u mem_activity_acc=%u xgmi_rd0=%lu fw_ts=%lu accum_ctr=%lu\n", m.gfx_activity_acc, m.mem_activity_acc, (unsigned long)m.xgmi_read_data_acc[0], (unsigned long)m.firmware_timestamp, (unsigned long)m.accumulation_counter);
      // Poll-rate probe: how fast can we read gpu_metrics?
      auto t0 = std::chrono::steady_clock::now();
      int n = 200; uint64_t last_ts = 0; int changes = 0;
      for (int i = 0; i < n; ++i) { amdsmi_get_gpu_metrics_info(h, &m); if (m.firmware_timestamp != last_ts) { changes++; last_ts = m.firmware_timestamp; } }
      double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
      std::printf("  gpu_metrics read: %.1f us/call, fw timestamp changed %d/%d\n", us, changes, n);
      t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < n; ++i) amdsmi_get_gpu_vram_usage(h, &v);
      us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
      std::printf("  vram_usage read: %.1f us/call\n", us);
      t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < n; ++i) amdsmi_get_power_info(h, &pw);
      us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
      std::printf("  power_info read: %.1f us/call\n", us);
    }
  }
  amdsmi_shut_down();
  return 0;
}
