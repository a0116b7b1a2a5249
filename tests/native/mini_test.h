// Minimal self-registering test harness for the native C API tests (the
// reference vendors googletest; we need only registration + checks).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#pragma once

#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

namespace mini_test {

struct Case {
  const char *name;
  std::function<void()> fn;
};

inline std::vector<Case> &registry() {
  static std::vector<Case> r;
  return r;
}

inline int &failures() {
  static int f = 0;
  return f;
}

struct Registrar {
  Registrar(const char *name, std::function<void()> fn) {
    registry().push_back({name, std::move(fn)});
  }
};

inline int run_all(int argc, char **argv) {
  const char *filter = nullptr;
  for (int i = 1; i < argc; i++) {
    if (std::strcmp(argv[i], "--list") == 0) {
      for (auto &c : registry()) std::printf("%s\n", c.name);
      return 0;
    }
    filter = argv[i];
  }
  int ran = 0, failed_cases = 0;
  for (auto &c : registry()) {
    if (filter && !std::strstr(c.name, filter)) continue;
    const int before = failures();
    c.fn();
    ran++;
    const bool ok = failures() == before;
    failed_cases += ok ? 0 : 1;
    std::printf("[%s] %s\n", ok ? "  OK  " : " FAIL ", c.name);
  }
  std::printf("%d case(s), %d failed\n", ran, failed_cases);
  return failed_cases ? 1 : 0;
}

}  // namespace mini_test

#define TEST_CASE(name)                                                 \
  static void name();                                                   \
  static mini_test::Registrar name##_registrar(#name, name);            \
  static void name()

#define CHECK(cond)                                                     \
  do {                                                                  \
    if (!(cond)) {                                                      \
      std::printf("  %s:%d: CHECK(%s) failed\n", __FILE__, __LINE__,    \
                  #cond);                                               \
      mini_test::failures()++;                                          \
    }                                                                   \
  } while (0)

#define CHECK_EQ(a, b)                                                  \
  do {                                                                  \
    if (!((a) == (b))) {                                                \
      std::printf("  %s:%d: CHECK_EQ(%s, %s) failed\n", __FILE__,       \
                  __LINE__, #a, #b);                                    \
      mini_test::failures()++;                                          \
    }                                                                   \
  } while (0)

#define CHECK_NEAR(a, b, tol)                                           \
  do {                                                                  \
    const double va_ = (a), vb_ = (b);                                  \
    if (!(std::fabs(va_ - vb_) <= (tol))) {                             \
      std::printf("  %s:%d: |%s - %s| = |%.9g - %.9g| > %g\n", __FILE__, \
                  __LINE__, #a, #b, va_, vb_, double(tol));             \
      mini_test::failures()++;                                          \
    }                                                                   \
  } while (0)
