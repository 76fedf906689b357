// Device-resident circular buffer: the MI355X replacement for cuda_buffer (reference
// runtime/include/gnuradio/cudabuffer.hpp:11-86, runtime/lib/cudabuffer.cu:17-183).
//
//  * storage: one HIP-VMM allocation mapped twice back to back (nsh_ring_alloc), so a
//    span starting anywhere is contiguous and nothing is ever mirror-copied (the
//    reference copies every written byte a second time and syncs, cudabuffer.cu:116-176);
//  * ordering: stream-ordered, never host-synchronised in steady state. post_write records
//    an event on the writer's stream and read_info makes a reader on a different stream
//    wait for it (hipStreamWaitEvent); post_read/write_info do the same for slot reuse.
//    Writer and reader on one partition stream need neither;
//  * H2D: host writer fills a pinned ring, post_write enqueues the copy on the buffer's
//    own stream; D2H: post_write enqueues the copy on the writer's stream and a host
//    reader sees items as their copy events complete (it blocks on the oldest pending
//    copy only when nothing else is readable);
//  * _total_read/_total_written are maintained (cuda_buffer never updates them,
//    cudabuffer.cu:107-176) and copy_items is an async device copy (the reference does a
//    host memcpy on device pointers, cudabuffer.cu:179-183).
#pragma once
#include <deque>
#include <gnuradio/buffer.hpp>
#include <utility>
#include <vector>

namespace gr {

enum class hip_buffer_type { D2D, H2D, D2H };

class hip_buffer_properties : public buffer_properties
{
public:
    explicit hip_buffer_properties(hip_buffer_type t, int device = -1) : _t(t), _dev(device) {}
    hip_buffer_type buffer_type() const { return _t; }
    int device() const { return _dev; } // -1: the creating thread's current device
    static std::shared_ptr<buffer_properties> make(hip_buffer_type t, int device = -1)
    {
        return std::make_shared<hip_buffer_properties>(t, device);
    }

private:
    hip_buffer_type _t;
    int _dev;
};

class hip_buffer : public buffer
{
public:
    using sptr = std::shared_ptr<hip_buffer>;
    static buffer_sptr make(size_t num_items, size_t item_size, std::shared_ptr<buffer_properties> props);
    hip_buffer(size_t num_items, size_t item_size, hip_buffer_type type, int device);
    ~hip_buffer() override;

    void* read_ptr() override;
    void* write_ptr() override;
    bool read_info(buffer_info_t& info) override;
    bool write_info(buffer_info_t& info) override;
    void post_read(int num_items) override;
    void post_write(int num_items) override;
    void copy_items(std::shared_ptr<buffer> from, int nitems) override;

    size_t capacity() const { return _cap; }
    size_t item_size() const { return _isz; }
    hip_buffer_type buffer_type() const { return _btype; }
    bool double_mapped() const { return _dm; }
    int device() const { return _dev; }
    void* device_base() const { return _dbase; } // ring start (mapped twice)
    void reset_flags() override;
    void discard_unread() override;

private:
    size_t readable_locked();
    void poll_pending_locked(bool block_if_empty);
    void* take_event();
    void wait_peer(void* event, void* peer_stream);

    hip_buffer_type _btype;
    int _dev;
    size_t _cap;  // items
    size_t _isz;  // bytes per item
    bool _dm = false;
    uint8_t* _dbase = nullptr; // device ring
    uint8_t* _hbase = nullptr; // pinned host ring (H2D / D2H)
    void* _cstream = nullptr;  // H2D copy stream

    void* _ev_written = nullptr; void* _writer_stream = nullptr; bool _w_rec = false;
    void* _ev_read = nullptr;    void* _reader_stream = nullptr; bool _r_rec = false;

    // in-flight host<->device copies: (event, total index they complete)
    std::deque<std::pair<void*, uint64_t>> _pending;
    std::vector<void*> _event_pool;
    uint64_t _copied = 0; // H2D: host slots whose copy finished; D2H: items visible on host
};

} // namespace gr

#define HIP_BUFFER_ARGS_H2D gr::hip_buffer::make, gr::hip_buffer_properties::make(gr::hip_buffer_type::H2D)
#define HIP_BUFFER_ARGS_D2H gr::hip_buffer::make, gr::hip_buffer_properties::make(gr::hip_buffer_type::D2H)
#define HIP_BUFFER_ARGS_D2D gr::hip_buffer::make, gr::hip_buffer_properties::make(gr::hip_buffer_type::D2D)
