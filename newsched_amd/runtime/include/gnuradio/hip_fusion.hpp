// Elementwise fusion for the GPU scheduler domain. Not in the reference (its blocks each
// launch and sync per work() call, blocklib/cuda/lib/copy.cpp:49-58); here a device block
// whose work() is a per-sample complex map y = x·k_1·…·k_m (copy: m = 0) says so by
// implementing elementwise_cc, and scheduler_hip rewrites every maximal chain of such
// blocks joined by device-to-device edges into ONE block that makes a single pass over HBM
// (the same per-stage rounding, so results are bit-identical to the unfused chain).
//
// What fusion changes, observably: the chain's interior edges get no buffer and the
// interior blocks' work() is not called (their nitems counters stay 0); the fused block
// reads the head's input edge and writes the tail's output edge, whose port connections
// are rewired to it. Tags pass through unchanged (every stage is 1:1 with the same
// propagation policy; chains with mixed policies are not fused).
#pragma once
#include <gnuradio/flat_graph.hpp>
#include <gnuradio/types.hpp>
#include <vector>

namespace gr {
namespace hip {

class elementwise_cc
{
public:
    virtual ~elementwise_cc() = default;
    // Append this block's stages (complex multipliers, applied in order) to `ks` and
    // return true; return false if this instance is not a complex map (e.g. a float
    // specialisation), which makes it a chain boundary.
    virtual bool elementwise_stages(std::vector<gr_complex>& ks) const = 0;
};

struct fusion_result {
    flat_graph_sptr graph;            // the rewritten partition (== input if nothing fused)
    std::vector<block_sptr> fused;    // the blocks that replaced chains
    std::vector<std::vector<block_sptr>> chains; // fused[i] replaced chains[i]
    // Port links the pass changed on the user's blocks (directed: first->connect/disconnect
    // (second)); undo() restores the graph's original links, so the same flowgraph can be
    // initialized again (validate, partition) with or without fusion.
    std::vector<std::pair<port_sptr, port_sptr>> cut, added;
    void undo()
    {
        for (auto it = added.rbegin(); it != added.rend(); ++it) it->first->disconnect(it->second);
        for (auto it = cut.rbegin(); it != cut.rend(); ++it) it->first->connect(it->second);
        added.clear();
        cut.clear();
    }
};

// Stages per fused block (the fused kernel's limit); longer chains become several blocks.
constexpr size_t max_fused_stages = 16;

// The pass (host logic only; touches no device). A chain is >= 2 elementwise_cc blocks,
// each with one input and one output stream port, linked by edges that are the only edge
// of their output port and carry no custom buffer or a hip_buffer of type D2D.
fusion_result fuse_elementwise_cc(flat_graph_sptr fg);

// Channelizer pass: fft_vcc(forward, 1024) -> multiply_const_vcc(w, 1024) -> fft_vcc(inverse,
// 1024), linked as above (single D2D edges, same tag policy), becomes ONE channelizer_vcc(w):
// the spectrum stays in registers (one HBM pass instead of three) and, with the same butterfly
// and product rounding in k_chan1024 as in the three kernels, the output is bit-identical.
fusion_result fuse_channelizer(flat_graph_sptr fg);

// FIR-chain pass: fir_filter_ccf blocks linked as above (single D2D edges, one input edge each,
// same tag policy; AUTO algorithm, no preloaded history) are cut into runs of >= 2 stages whose
// total decimation is 8 or 16 (the longest such run from each position) and each run becomes
// ONE fir_filter_cascade_ccf: one HBM pass over the input instead of one per stage, results
// within fp32 transform rounding of the staged chain (not bit-identical: the composite filter is
// applied by polyphase FFT). scheduler_hip::set_fir_fusion(false) turns it off.
fusion_result fuse_fir_cascade(flat_graph_sptr fg);

} // namespace hip
} // namespace gr
