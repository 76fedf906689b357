// Buffer plugin interface (reference runtime/include/gnuradio/buffer.hpp:18-223).
//
// A buffer is the edge between one writer port and one reader port. Executors ask it how
// many items can be read/written (read_info/write_info), hand read_ptr()/write_ptr()
// spans to work(), then advance it (post_read/post_write). Subclasses: vmcirc_buffer
// (host, double-mapped), hip_buffer (device ring; gr/hip_buffer.hpp), domain adapters.
//
// Additions over the reference, all non-virtual bookkeeping in the base class:
//   * writer_done()/reader_done() let executors finish a flowgraph by draining instead of
//     the reference's fixed 100 ms sleep (runtime/lib/flowgraph_monitor.cpp:27);
//   * reset() rewinds the completion flags for a restarted flowgraph.
#pragma once
#include <algorithm>
#include <atomic>
#include <functional>
#include <gnuradio/tag.hpp>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace gr {

struct buffer_info_t {
    void* ptr;
    int n_items;      // items readable / writable now
    size_t item_size;
    int total_items;  // reference field (int, as there); see total_read()/total_written()
};

class buffer
{
public:
    virtual ~buffer() = default;

    virtual void* read_ptr() = 0;
    virtual void* write_ptr() = 0;
    virtual bool read_info(buffer_info_t& info) = 0;
    virtual bool write_info(buffer_info_t& info) = 0;
    virtual void post_read(int num_items) = 0;
    virtual void post_write(int num_items) = 0;
    // Duplicate nitems just written into `from` (the first buffer of a fan-out port) into
    // this buffer's write span (graph_executor fan-out, reference graph_executor.cpp:188-200).
    virtual void copy_items(std::shared_ptr<buffer> from, int nitems) = 0;

    // ---- tags (host side) ----
    // The buffer whose tag list and counters these calls use: this one, or for a domain
    // adapter the edge buffer it stands for (so tags cross in-process domain boundaries).
    virtual buffer* tag_target() { return this; }

    virtual std::vector<tag_t> get_tags(unsigned int num_items)
    {
        if (auto* t = tag_target(); t != this) return t->get_tags(num_items);
        std::lock_guard<std::mutex> g(_buf_mutex);
        std::vector<tag_t> r;
        for (auto& t : _tags)
            if (t.offset >= _total_read && t.offset < _total_read + num_items) r.push_back(t);
        return r;
    }
    virtual void add_tags(unsigned int num_items, std::vector<tag_t>& tags)
    {
        if (auto* t = tag_target(); t != this) return t->add_tags(num_items, tags);
        std::lock_guard<std::mutex> g(_buf_mutex);
        for (auto& t : tags)
            if (t.offset + num_items >= _total_written && t.offset < _total_written) _tags.push_back(t);
    }
    bool has_tags()
    {
        auto* t = tag_target();
        std::lock_guard<std::mutex> g(t->_buf_mutex);
        return !t->_tags.empty();
    }
    std::vector<tag_t> tags()
    {
        auto* t = tag_target();
        std::lock_guard<std::mutex> g(t->_buf_mutex);
        return t->_tags;
    }
    std::vector<tag_t> tags_in_window(uint64_t item_start, uint64_t item_end)
    {
        if (auto* t = tag_target(); t != this) return t->tags_in_window(item_start, item_end);
        std::lock_guard<std::mutex> g(_buf_mutex);
        std::vector<tag_t> r;
        for (auto& t : _tags)
            if (t.offset >= _total_read + item_start && t.offset < _total_read + item_end) r.push_back(t);
        return r;
    }
    void add_tag(tag_t tag)
    {
        if (auto* t = tag_target(); t != this) return t->add_tag(std::move(tag));
        std::lock_guard<std::mutex> g(_buf_mutex);
        _tags.push_back(std::move(tag));
    }
    void add_tag(uint64_t offset, pmtf::pmt_sptr key, pmtf::pmt_sptr value, pmtf::pmt_sptr srcid = nullptr)
    {
        add_tag(tag_t(offset, std::move(key), std::move(value), std::move(srcid)));
    }
    // Copy tags of `in` that fall in the window this block is about to write.
    void propagate_tags(std::shared_ptr<buffer> in, int n_consumed)
    {
        if (auto* t = tag_target(); t != this) return t->propagate_tags(std::move(in), n_consumed);
        std::vector<tag_t> src = in->tags();
        std::lock_guard<std::mutex> g(_buf_mutex);
        for (auto& t : src)
            if (t.offset >= _total_written && t.offset < _total_written + (uint64_t)n_consumed) _tags.push_back(t);
    }
    void prune_tags(int n_consumed)
    {
        if (auto* t = tag_target(); t != this) return t->prune_tags(n_consumed);
        std::lock_guard<std::mutex> g(_buf_mutex);
        const uint64_t lim = _total_read + (uint64_t)n_consumed;
        _tags.erase(std::remove_if(_tags.begin(), _tags.end(), [lim](const tag_t& t) { return t.offset < lim; }),
                    _tags.end());
    }

    void set_name(const std::string& n) { _name = n; }
    std::string name() const { return _name; }
    std::string type() const { return _type; }
    // Absolute item counters (tag offsets are relative to these); a domain adapter reports
    // those of the edge buffer it stands for.
    uint64_t total_written()
    {
        auto* t = tag_target();
        return t == this ? _total_written : t->total_written();
    }
    uint64_t total_read()
    {
        auto* t = tag_target();
        return t == this ? _total_read : t->total_read();
    }

    // ---- completion bookkeeping (drain-correct termination) ----
    // virtual so domain adapters can forward them to the buffer they stand for
    virtual void set_writer_done() { _writer_done.store(true); }
    virtual void set_reader_done() { _reader_done.store(true); }
    virtual bool writer_done() const { return _writer_done.load(); }
    virtual bool reader_done() const { return _reader_done.load(); }
    virtual void reset_flags()
    {
        _writer_done.store(false);
        _reader_done.store(false);
    }
    // A restarted flowgraph is a new run: items the previous run wrote but nobody read (a
    // decimator's input remainder below one output, a source that ran ahead of a head) are
    // dropped with their tags, so the next run's stream starts at its first item. Called from
    // prepare_run() with every thread of the previous run finished and every stream drained.
    // Default: nothing kept (buffers that hold no items of their own, e.g. remote adapters).
    virtual void discard_unread() {}

protected:
    void set_type(const std::string& t) { _type = t; }
    std::string _name;
    std::string _type;
    uint64_t _total_read = 0;
    uint64_t _total_written = 0;
    // the discard_unread() bookkeeping shared by the ring buffers (caller holds _buf_mutex)
    void drop_unread_locked()
    {
        _total_read = _total_written;
        _tags.erase(std::remove_if(_tags.begin(), _tags.end(), [this](const tag_t& t) { return t.offset < _total_read; }),
                    _tags.end());
    }
    std::mutex _buf_mutex;
    std::vector<tag_t> _tags;

private:
    std::atomic<bool> _writer_done{ false };
    std::atomic<bool> _reader_done{ false };
};

using buffer_sptr = std::shared_ptr<buffer>;

// Base for per-buffer-type construction options passed through the factory.
class buffer_properties
{
public:
    buffer_properties() = default;
    virtual ~buffer_properties() = default;
};

using buffer_factory_function =
    std::function<std::shared_ptr<buffer>(size_t num_items, size_t item_size, std::shared_ptr<buffer_properties>)>;

} // namespace gr
