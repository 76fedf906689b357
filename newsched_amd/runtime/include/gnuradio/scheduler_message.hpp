// Scheduler thread messages (reference runtime/include/gnuradio/scheduler_message.hpp:8-64).
#pragma once
#include <cstdint>
#include <functional>
#include <gnuradio/pmtf.hpp>
#include <memory>

namespace gr {

enum class scheduler_action_t { DONE, NOTIFY_OUTPUT, NOTIFY_INPUT, NOTIFY_ALL, EXIT };
enum class scheduler_message_t { SCHEDULER_ACTION, MSGPORT_MESSAGE };

class scheduler_message
{
public:
    explicit scheduler_message(scheduler_message_t t) : _type(t) {}
    virtual ~scheduler_message() = default;
    scheduler_message_t type() const { return _type; }
    void set_blkid(int64_t id) { _blkid = id; }
    int64_t blkid() const { return _blkid; }

private:
    scheduler_message_t _type;
    int64_t _blkid = -1;
};
using scheduler_message_sptr = std::shared_ptr<scheduler_message>;

class scheduler_action : public scheduler_message
{
public:
    scheduler_action(scheduler_action_t a, uint32_t blkid = 0)
        : scheduler_message(scheduler_message_t::SCHEDULER_ACTION), _action(a)
    {
        set_blkid(int64_t{ blkid });
    }
    scheduler_action_t action() const { return _action; }

private:
    scheduler_action_t _action;
};
using scheduler_action_sptr = std::shared_ptr<scheduler_action>;

using message_port_callback_fcn = std::function<void(pmtf::pmt_sptr)>;

class msgport_message : public scheduler_message
{
public:
    msgport_message(pmtf::pmt_sptr msg, message_port_callback_fcn cb)
        : scheduler_message(scheduler_message_t::MSGPORT_MESSAGE), _msg(std::move(msg)), _cb(std::move(cb))
    {
    }
    void set_callback(message_port_callback_fcn cb) { _cb = std::move(cb); }
    message_port_callback_fcn callback() const { return _cb; }
    pmtf::pmt_sptr message() const { return _msg; }

private:
    pmtf::pmt_sptr _msg;
    message_port_callback_fcn _cb;
};
using msgport_message_sptr = std::shared_ptr<msgport_message>;

} // namespace gr
