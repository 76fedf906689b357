// Executor status vocabulary (reference runtime/include/gnuradio/executor.hpp).
#pragma once
#include <gnuradio/logging.hpp>
#include <string>

namespace gr {
enum class executor_state { WORKING, DONE, FLUSHED, EXIT };
enum class executor_iteration_status {
    READY,           // made progress
    READY_NO_OUTPUT, // consumed without producing
    BLKD_IN,         // waiting for input
    BLKD_OUT,        // waiting for output space
    DONE,            // finished for this run
};
class executor
{
public:
    explicit executor(const std::string& name) : _name(name)
    {
        _logger = logging::get_logger(name, "default");
        _debug_logger = logging::get_logger(name + "_dbg", "debug");
    }
    virtual ~executor() = default;

protected:
    std::string _name;
    logger_sptr _logger;
    logger_sptr _debug_logger;
};
} // namespace gr
