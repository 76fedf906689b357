// Logging restated as compile-time no-ops. The reference builds spdlog loggers from
// ~/.gnuradio/config.yml and they are nullptr without it (runtime/lib/logging.cpp:91-136),
// so its hot-loop GR_LOG_DEBUG calls (schedulers/mt/lib/graph_executor.cpp:29-30, ...)
// cost nothing by default; here they cost nothing always. NEWSCHED_LOG=1 prints
// INFO/WARN/ERROR lines to stderr for debugging.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>

namespace gr {
struct logger {
    std::string name;
};
using logger_sptr = std::shared_ptr<logger>;
namespace logging {
inline logger_sptr get_logger(const std::string& name, const std::string& /*cfg*/)
{
    return std::make_shared<logger>(logger{ name });
}
inline bool enabled()
{
    static const bool on = [] {
        const char* e = std::getenv("NEWSCHED_LOG");
        return e && *e == '1';
    }();
    return on;
}
} // namespace logging
} // namespace gr

#define GR_LOG_TRACE(l, ...) ((void)0)
#define GR_LOG_DEBUG(l, ...) ((void)0)
#define gr_log_debug(l, ...) ((void)0)
#define GR_LOG_INFO(l, msg)                                                              \
    do {                                                                                 \
        if (::gr::logging::enabled() && (l))                                             \
            std::fprintf(stderr, "[INFO] %s: %s\n", (l)->name.c_str(), std::string(msg).c_str()); \
    } while (0)
#define GR_LOG_WARN(l, msg)                                                              \
    do {                                                                                 \
        if (::gr::logging::enabled() && (l))                                             \
            std::fprintf(stderr, "[WARN] %s: %s\n", (l)->name.c_str(), std::string(msg).c_str()); \
    } while (0)
#define GR_LOG_ERROR(l, msg)                                                             \
    do {                                                                                 \
        if (l) std::fprintf(stderr, "[ERROR] %s: %s\n", (l)->name.c_str(), std::string(msg).c_str()); \
    } while (0)
