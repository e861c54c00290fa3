// Where the per-call time of a small struct_pack::gpu call goes: the single
// steps of the small-call path (copies, launches, syncs) timed on their own,
// then whole serialize / deserialize calls, on the thread's stream.
#include <chrono>
#include <cstring>
#include <cstdio>
#include <string>
#include <tuple>
#include <vector>

#include "ylt/struct_pack_gpu.hpp"

namespace gp = struct_pack::gpu;
using clk = std::chrono::steady_clock;

template <typename F>
double us(F f, int n = 2000) {
  for (int i = 0; i < 50; ++i) f();
  const auto t0 = clk::now();
  for (int i = 0; i < n; ++i) f();
  return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / n;
}

struct Person {
  int64_t id;
  std::string name;
  int age;
  double salary;
};

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  void *s = gp::device::thread_stream();
  void *d = nullptr, *h = nullptr;
  gp::device::check(spk_device_alloc(&d, 1 << 20), "alloc");
  gp::device::check(spk_host_alloc_pinned(&h, 1 << 20), "pinned");
  std::printf("sync alone              %7.2f us\n", us([&] { gp::device::sync(s); }));
  std::printf("H2D 64 B + sync         %7.2f us\n", us([&] {
                gp::device::copy(d, h, 64, SPK_COPY_H2D, s);
                gp::device::sync(s);
              }));
  std::printf("D2H 4 KiB + sync        %7.2f us\n", us([&] {
                gp::device::copy(h, d, 4096, SPK_COPY_D2H, s);
                gp::device::sync(s);
              }));
  std::printf("H2D + D2H + sync        %7.2f us\n", us([&] {
                gp::device::copy(d, h, 64, SPK_COPY_H2D, s);
                gp::device::copy((char *)h + 4096, (char *)d + 4096, 4096, SPK_COPY_D2H, s);
                gp::device::sync(s);
              }));
  const std::tuple<int, int> args{40, 2};
  const int ret = 42;
  const Person p{7, "a person's name", 40, 1234.5};
  std::printf("serialize(int)          %7.2f us\n",
              us([&] { (void)gp::serialize<std::string>(ret); }));
  std::printf("serialize(tuple<int,int>) %5.2f us\n",
              us([&] { (void)gp::serialize<std::string>(args); }));
  std::printf("serialize(Person)       %7.2f us\n",
              us([&] { (void)gp::serialize<std::string>(p); }));
  const std::string wa = gp::serialize<std::string>(args), wp = gp::serialize<std::string>(p);
  std::printf("deserialize(tuple)      %7.2f us\n", us([&] {
                std::tuple<int, int> t;
                (void)gp::deserialize_to(t, wa);
              }));
  std::printf("deserialize(Person)     %7.2f us\n", us([&] {
                Person q;
                (void)gp::deserialize_to(q, wp);
              }));
  spk_trace_enable(1);
  spk_trace_reset();
  for (int i = 0; i < 10; ++i) {
    Person q;
    (void)gp::deserialize_to(q, wp);
    (void)gp::serialize<std::string>(p);
  }
  std::vector<char> buf(1 << 16);
  spk_trace_read(buf.data(), buf.size());
  std::printf("launches over 10 Person decode+encode calls:\n%s\n", buf.data());
  return 0;
}
