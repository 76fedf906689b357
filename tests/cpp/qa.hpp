// Minimal test harness standing in for gtest (absent here). TEST(a, b)
// registers a case; EXPECT_* record failures; main() runs the cases named on the
// command line (or all) and returns nonzero on any failure.
#pragma once
#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>
#include <cstring>
#include <functional>
#include <sstream>
#include <string>
#include <vector>

namespace qa {
struct test_case {
    std::string name;
    std::function<void()> fn;
};
inline std::vector<test_case>& registry()
{
    static std::vector<test_case> r;
    return r;
}
inline int& failures()
{
    static int f = 0;
    return f;
}
struct reg {
    reg(const char* a, const char* b, std::function<void()> f) { registry().push_back({ std::string(a) + "." + b, f }); }
};
inline void fail(const char* file, int line, const std::string& what)
{
    ++failures();
    std::fprintf(stderr, "  FAIL %s:%d: %s\n", file, line, what.c_str());
}
} // namespace qa

#define TEST(A, B)                                             \
    static void A##_##B##_impl();                              \
    static qa::reg A##_##B##_reg(#A, #B, A##_##B##_impl);      \
    static void A##_##B##_impl()

#define EXPECT_TRUE(c)                                          \
    do {                                                        \
        if (!(c)) qa::fail(__FILE__, __LINE__, #c);             \
    } while (0)
#define EXPECT_FALSE(c) EXPECT_TRUE(!(c))
#define EXPECT_EQ(a, b)                                                         \
    do {                                                                        \
        if (!((a) == (b))) qa::fail(__FILE__, __LINE__, #a " == " #b);          \
    } while (0)
#define ASSERT_TRUE(c)                                          \
    do {                                                        \
        if (!(c)) {                                             \
            qa::fail(__FILE__, __LINE__, #c);                   \
            return;                                             \
        }                                                       \
    } while (0)

namespace qa {
inline const char*& current_name()
{
    static const char* n = "";
    return n;
}
// Watchdog: a case that hangs fails with its name instead of stalling the whole suite.
inline void on_alarm(int)
{
    const char* a = "\n  TIMEOUT in ";
    (void)!write(2, a, std::strlen(a));
    (void)!write(2, current_name(), std::strlen(current_name()));
    (void)!write(2, "\n", 1);
    _exit(3);
}
} // namespace qa

int main(int argc, char** argv)
{
    int run = 0;
    std::setvbuf(stdout, nullptr, _IOLBF, 0); // lines reach a pipe / file as they are printed
    const char* tmo = std::getenv("QA_CASE_TIMEOUT");
    const unsigned case_timeout = tmo ? (unsigned)std::atoi(tmo) : 240u;
    std::signal(SIGALRM, qa::on_alarm);
    for (auto& t : qa::registry()) {
        bool sel = argc < 2;
        for (int i = 1; i < argc; ++i)
            if (t.name.find(argv[i]) != std::string::npos) sel = true;
        if (!sel) continue;
        const int before = qa::failures();
        const auto t0 = std::chrono::steady_clock::now();
        qa::current_name() = t.name.c_str();
        alarm(case_timeout);
        try {
            t.fn();
        } catch (const std::exception& e) {
            qa::fail(__FILE__, __LINE__, std::string("exception: ") + e.what());
        }
        alarm(0);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("[%s] %s (%.3f s)\n", qa::failures() == before ? " OK " : "FAIL", t.name.c_str(), s);
        ++run;
    }
    std::printf("%d test(s), %d failure(s)\n", run, qa::failures());
    return qa::failures() ? 1 : 0;
}
