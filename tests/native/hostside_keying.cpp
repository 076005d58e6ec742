// CPU test of the forward's host-side resource keying (csrc/hostside.h)
// against a mock device API: the resources a call uses belong to the device
// of its stream, whatever device the thread has current, and the thread's
// current device is restored afterwards.  Built and run by
// tests/test_host.py::test_host_resources_keyed_by_stream_device.
#include <cstdio>
#include <cstdlib>
#include <map>

#include "hostside.h"

static int g_cur = 0;                    // the thread's current device
static std::map<void *, int> g_streams;  // stream -> device
static int g_sets = 0;

struct MockApi {
  static int get_device(int *d) { *d = g_cur; return 0; }
  static int set_device(int d) { g_cur = d; ++g_sets; return 0; }
  static int stream_device(void *s, int *d) {
    auto it = g_streams.find(s);
    if (it == g_streams.end()) return 1;
    *d = it->second;
    return 0;
  }
};

struct Res {
  int uses = 0;
};

#define CHECK(c)                                                 \
  do {                                                           \
    if (!(c)) {                                                  \
      std::fprintf(stderr, "FAIL line %d: %s\n", __LINE__, #c);  \
      std::exit(1);                                              \
    }                                                            \
  } while (0)

// One "entry point": its resources are those of its stream's device.
static int call(std::map<int, Res> &all, void *stream) {
  rnnl::DeviceGuardT<MockApi> guard(rnnl::stream_device_of<MockApi>(stream));
  int dev = -1;
  Res *r = rnnl::current_device_entry<MockApi>(all, &dev);
  CHECK(r != nullptr);
  ++r->uses;
  return dev;
}

int main() {
  std::map<int, Res> all;
  int s3 = 0, s5 = 0;
  g_streams[&s3] = 3;
  g_streams[&s5] = 5;
  g_cur = 0;
  // a caller whose current device is 0 runs on a stream of device 3
  CHECK(call(all, &s3) == 3);
  CHECK(g_cur == 0);  // restored
  CHECK(all.count(3) == 1 && all[3].uses == 1 && all.count(0) == 0);
  // another device's stream: its own resources
  CHECK(call(all, &s5) == 5);
  CHECK(all[5].uses == 1 && all[3].uses == 1 && g_cur == 0);
  // a null stream is the current device's
  g_cur = 3;
  const int sets = g_sets;
  CHECK(call(all, nullptr) == 3);
  CHECK(all[3].uses == 2 && g_sets == sets);  // already current: no device switch
  // an unknown stream (device unreadable): no switch, the current device's
  g_cur = 5;
  int other = 0;
  void *bogus = &other;
  CHECK(rnnl::stream_device_of<MockApi>(bogus) == -1);
  CHECK(call(all, bogus) == 5 && all[5].uses == 2 && g_cur == 5);
  std::printf("ok\n");
  return 0;
}
