// GPU-box probe: cost of one pread of the SMU metrics table (sysfs gpu_metrics) in a
// process that touches nothing else (no HIP, no amd-smi). Run it as several fresh
// processes to see whether the fast / slow read states (BASELINE.md "run-to-run
// variance") exist without our runtime, and whether a busy GPU changes them.
#include <fcntl.h>
#include <glob.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2000;
  glob_t g{};
  if (glob("/sys/class/drm/card*/device/gpu_metrics", 0, nullptr, &g) != 0 || g.gl_pathc == 0) {
    std::printf("no gpu_metrics\n");
    return 1;
  }
  const int fd = ::open(g.gl_pathv[0], O_RDONLY | O_CLOEXEC);
  if (fd < 0) return 1;
  std::vector<unsigned char> buf(4096);
  std::vector<double> us;
  us.reserve(n);
  for (int i = 0; i < n; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    if (::pread(fd, buf.data(), buf.size(), 0) <= 0) return 1;
    us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  std::sort(us.begin(), us.end());
  std::printf("%s cpu %d: pread p10 %.1f p50 %.1f p90 %.1f us\n", g.gl_pathv[0], sched_getcpu(), us[n / 10], us[n / 2],
              us[9 * n / 10]);
  ::close(fd);
  globfree(&g);
  return 0;
}
