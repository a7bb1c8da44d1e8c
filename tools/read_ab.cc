// Host file-read A/B for the trainer's corpus load (c5: 2.6 GB text file):
// (a) single read() into a zero-filled std::string (the round-2 reader),
// (b) 16 threads pread() 64 MB pieces into an uninitialized buffer,
// (c) mmap(MAP_POPULATE) of the file, then a parallel byte sum (touch),
// (d) 16 threads first-touch memcpy of the buffer into a fresh malloc'ed one.
//   g++ -O2 -std=c++17 -pthread tools/read_ab.cc -o /tmp/read_ab && /tmp/read_ab FILE
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

static double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  const char *fn = argv[1];
  struct stat sb;
  stat(fn, &sb);
  const size_t size = sb.st_size;
  const int T = 16;
  double t0 = Now();
  {
    std::ifstream is(fn, std::ios::binary);
    std::string data;
    data.resize(size);
    is.read(&data[0], size);
    printf("(a) single read into zeroed string: %.3f s\n", Now() - t0);
  }
  t0 = Now();
  std::unique_ptr<char[]> buf(new char[size]);
  {
    int fd = open(fn, O_RDONLY);
    const size_t P = 64ull << 20, pieces = (size + P - 1) / P;
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&]() {
        for (size_t k = next++; k < pieces; k = next++) {
          size_t o = k * P, e = std::min(size, o + P);
          while (o < e) {
            ssize_t r = pread(fd, buf.get() + o, e - o, o);
            if (r <= 0) break;
            o += r;
          }
        }
      });
    for (auto &x : th) x.join();
    close(fd);
    printf("(b) 16-thread pread into new char[]: %.3f s\n", Now() - t0);
  }
  t0 = Now();
  {
    int fd = open(fn, O_RDONLY);
    void *m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
    double t1 = Now();
    std::vector<std::thread> th;
    std::vector<uint64_t> sum(T);
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        const unsigned char *p = static_cast<const unsigned char *>(m);
        uint64_t s = 0;
        for (size_t k = size * t / T; k < size * (t + 1) / T; k += 64) s += p[k];
        sum[t] = s;
      });
    for (auto &x : th) x.join();
    printf("(c) mmap populate %.3f s + parallel touch %.3f s\n", t1 - t0, Now() - t1);
    munmap(m, size);
    close(fd);
  }
  t0 = Now();
  {
    std::unique_ptr<char[]> dst(new char[size]);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        const size_t a = size * t / T, b = size * (t + 1) / T;
        memcpy(dst.get() + a, buf.get() + a, b - a);
      });
    for (auto &x : th) x.join();
    printf("(d) 16-thread first-touch memcpy: %.3f s\n", Now() - t0);
  }
  return 0;
}
