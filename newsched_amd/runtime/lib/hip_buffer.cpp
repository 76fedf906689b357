// Device-resident ring buffer (see hip_buffer.hpp for the design and the reference
// behaviour it replaces).
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/hip_context.hpp>

#include <algorithm>
#include <cstring>
#include <numeric>
#include <stdexcept>

#include "nsh_hip.h"

namespace gr {

using hip::check;

buffer_sptr hip_buffer::make(size_t num_items, size_t item_size, std::shared_ptr<buffer_properties> props)
{
    auto p = std::dynamic_pointer_cast<hip_buffer_properties>(props);
    if (!p) throw std::runtime_error("Failed to cast buffer properties to hip_buffer_properties");
    const int dev = p->device() >= 0 ? p->device() : hip::current_device();
    return std::make_shared<hip_buffer>(num_items, item_size, p->buffer_type(), dev);
}

hip_buffer::hip_buffer(size_t num_items, size_t item_size, hip_buffer_type type, int device)
    : _btype(type), _dev(device), _isz(item_size)
{
    if (item_size == 0) throw std::invalid_argument("hip_buffer: item_size 0");
    // ring bytes a multiple of the 4 KiB VMM granule so the second mapping lands on an
    // item boundary
    const size_t unit = std::lcm<size_t>(4096, item_size) / item_size;
    _cap = (std::max<size_t>(num_items, 2) + unit - 1) / unit * unit;
    void* base = nullptr;
    size_t actual = 0;
    int dm = 0;
    check(nsh_ring_alloc(_dev, _cap * _isz, &base, &actual, &dm), "hip_buffer: ring alloc");
    _dbase = (uint8_t*)base;
    _dm = dm != 0;
    if (actual != _cap * _isz) {
        if (actual % _isz == 0)
            _cap = actual / _isz;
        else
            _dm = false; // mirror would not start on an item boundary: cap spans at wrap
    }
    if (_btype != hip_buffer_type::D2D) {
        void* h = nullptr;
        check(nsh_host_alloc(_cap * _isz, &h), "hip_buffer: pinned host ring");
        _hbase = (uint8_t*)h;
    }
    if (_btype == hip_buffer_type::H2D) check(nsh_stream_create(_dev, &_cstream), "hip_buffer: copy stream");
    check(nsh_event_create(&_ev_written), "hip_buffer: event");
    check(nsh_event_create(&_ev_read), "hip_buffer: event");
    set_type(std::string("hip_buffer_") +
             (_btype == hip_buffer_type::D2D ? "D2D" : _btype == hip_buffer_type::H2D ? "H2D" : "D2H"));
}

hip_buffer::~hip_buffer()
{
    if (_cstream) nsh_stream_sync(_cstream);
    for (auto& p : _pending) {
        nsh_event_sync(p.first);
        nsh_event_destroy(p.first);
    }
    for (void* e : _event_pool) nsh_event_destroy(e);
    if (_ev_written) nsh_event_destroy(_ev_written);
    if (_ev_read) nsh_event_destroy(_ev_read);
    if (_cstream) nsh_stream_destroy(_cstream);
    if (_dbase) nsh_ring_free(_dbase);
    if (_hbase) nsh_host_free(_hbase);
}

void* hip_buffer::read_ptr()
{
    uint8_t* b = _btype == hip_buffer_type::D2H ? _hbase : _dbase;
    return b + (_total_read % _cap) * _isz;
}

void* hip_buffer::write_ptr()
{
    uint8_t* b = _btype == hip_buffer_type::H2D ? _hbase : _dbase;
    return b + (_total_written % _cap) * _isz;
}

void* hip_buffer::take_event()
{
    if (!_event_pool.empty()) {
        void* e = _event_pool.back();
        _event_pool.pop_back();
        return e;
    }
    void* e = nullptr;
    check(nsh_event_create(&e), "hip_buffer: event");
    return e;
}

// Retire completed host<->device copies (FIFO). With block_first, first wait for the
// oldest one (the caller has nothing to do until it lands).
void hip_buffer::poll_pending_locked(bool block_first)
{
    if (block_first && !_pending.empty()) check(nsh_event_sync(_pending.front().first), "hip_buffer: copy wait");
    while (!_pending.empty()) {
        const int q = nsh_event_query(_pending.front().first);
        if (q < 0) check(-1, "hip_buffer: event query");
        if (q != 0) break;
        _copied = _pending.front().second;
        _event_pool.push_back(_pending.front().first);
        _pending.pop_front();
    }
}

void hip_buffer::wait_peer(void* event, void* peer_stream)
{
    void* s = hip::current_stream();
    if (peer_stream != s) check(nsh_stream_wait_event(s, event), "hip_buffer: stream wait");
}

bool hip_buffer::read_info(buffer_info_t& info)
{
    std::lock_guard<std::mutex> g(_buf_mutex);
    int64_t n;
    if (_btype == hip_buffer_type::D2H) {
        poll_pending_locked(false);
        if (_copied == _total_read && !_pending.empty()) poll_pending_locked(true);
        n = (int64_t)(_copied - _total_read);
        n = std::min<int64_t>(n, (int64_t)(_cap - _total_read % _cap)); // host ring wraps
    } else {
        n = (int64_t)(_total_written - _total_read);
        if (!_dm) n = std::min<int64_t>(n, (int64_t)(_cap - _total_read % _cap));
        if (n > 0 && _w_rec) wait_peer(_ev_written, _writer_stream);
    }
    info.ptr = read_ptr();
    info.n_items = (int)std::min<int64_t>(n, 0x7fffffff);
    info.item_size = _isz;
    info.total_items = (int)_total_read;
    return true;
}

bool hip_buffer::write_info(buffer_info_t& info)
{
    std::lock_guard<std::mutex> g(_buf_mutex);
    const int64_t used = (int64_t)(_total_written - _total_read);
    int64_t n = (int64_t)_cap - used - 1;
    n = std::min<int64_t>(n, (int64_t)_cap / 2);
    if (_btype == hip_buffer_type::H2D) {
        n = std::min<int64_t>(n, (int64_t)(_cap - _total_written % _cap)); // host ring wraps
        poll_pending_locked(false);
        auto host_free = [&] { return (int64_t)_cap - (int64_t)(_total_written - _copied); };
        if (n > 0 && host_free() <= 0 && !_pending.empty()) poll_pending_locked(true);
        n = std::min<int64_t>(n, host_free());
    } else {
        if (!_dm) n = std::min<int64_t>(n, (int64_t)(_cap - _total_written % _cap));
        if (n > 0 && _r_rec && _btype == hip_buffer_type::D2D) wait_peer(_ev_read, _reader_stream);
    }
    info.ptr = write_ptr();
    info.n_items = (int)std::max<int64_t>(0, std::min<int64_t>(n, 0x7fffffff));
    info.item_size = _isz;
    info.total_items = (int)_total_written;
    return true;
}

void hip_buffer::post_write(int num_items)
{
    if (num_items <= 0) return;
    std::lock_guard<std::mutex> g(_buf_mutex);
    const size_t off = (_total_written % _cap) * _isz;
    const size_t bytes = (size_t)num_items * _isz;
    switch (_btype) {
    case hip_buffer_type::D2D: {
        void* s = hip::current_stream();
        if (_reader_stream == nullptr || _reader_stream != s) {
            check(nsh_event_record(_ev_written, s), "hip_buffer: record write");
            _w_rec = true;
        }
        _writer_stream = s;
        break;
    }
    case hip_buffer_type::H2D: {
        if (_r_rec) check(nsh_stream_wait_event(_cstream, _ev_read), "hip_buffer: slot reuse wait");
        check(nsh_memcpy_async(_dbase + off, _hbase + off, bytes, NSH_H2D, _cstream), "hip_buffer: H2D copy");
        void* e = take_event();
        check(nsh_event_record(e, _cstream), "hip_buffer: record copy");
        _pending.emplace_back(e, _total_written + (uint64_t)num_items);
        check(nsh_event_record(_ev_written, _cstream), "hip_buffer: record write");
        _w_rec = true;
        _writer_stream = _cstream;
        break;
    }
    case hip_buffer_type::D2H: {
        void* s = hip::current_stream();
        const size_t first = std::min(bytes, _cap * _isz - off); // host ring is single-mapped
        check(nsh_memcpy_async(_hbase + off, _dbase + off, first, NSH_D2H, s), "hip_buffer: D2H copy");
        if (first < bytes)
            check(nsh_memcpy_async(_hbase, _dbase + off + first, bytes - first, NSH_D2H, s), "hip_buffer: D2H copy");
        void* e = take_event();
        check(nsh_event_record(e, s), "hip_buffer: record copy");
        _pending.emplace_back(e, _total_written + (uint64_t)num_items);
        _writer_stream = s;
        break;
    }
    }
    _total_written += (uint64_t)num_items;
}

void hip_buffer::post_read(int num_items)
{
    if (num_items <= 0) return;
    std::lock_guard<std::mutex> g(_buf_mutex);
    _total_read += (uint64_t)num_items;
    if (_btype != hip_buffer_type::D2H) {
        void* s = hip::current_stream();
        if (_writer_stream == nullptr || _writer_stream != s) {
            check(nsh_event_record(_ev_read, s), "hip_buffer: record read");
            _r_rec = true;
        }
        _reader_stream = s;
    }
}

void hip_buffer::copy_items(std::shared_ptr<buffer> from, int nitems)
{
    if (nitems <= 0) return;
    std::lock_guard<std::mutex> g(_buf_mutex);
    void* dst = write_ptr();
    const void* src = from->write_ptr();
    const size_t bytes = (size_t)nitems * _isz;
    auto hb = std::dynamic_pointer_cast<hip_buffer>(from);
    const bool src_host = !hb || hb->buffer_type() == hip_buffer_type::H2D;
    if (_btype == hip_buffer_type::H2D) {
        if (src_host) {
            std::memcpy(dst, src, bytes);
        } else {
            void* s = hip::current_stream();
            check(nsh_memcpy_async(dst, src, bytes, NSH_DEFAULT, s), "hip_buffer: copy_items");
            check(nsh_stream_sync(s), "hip_buffer: copy_items");
        }
        return;
    }
    check(nsh_memcpy_async(dst, src, bytes, NSH_DEFAULT, hip::current_stream()), "hip_buffer: copy_items");
}

void hip_buffer::reset_flags() { buffer::reset_flags(); }

void hip_buffer::discard_unread()
{
    std::lock_guard<std::mutex> g(_buf_mutex);
    while (!_pending.empty()) poll_pending_locked(true); // host<->device copies of the last run
    drop_unread_locked();
}

} // namespace gr
