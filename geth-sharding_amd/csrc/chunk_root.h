// Collation chunk root (sharding/collation.go:115-119 CalculateChunkRoot = types.DeriveSha over
// Chunks(body), core/types/derive_sha.go:32-41) on gfx950.
//
// The trie SHAPE depends only on N = len(body): keys are rlp(uint(i)) for i < N.  The host builds a
// "plan" per N once (cached in the context): every internal node of the Merkle-Patricia trie with
// its kind, height and where its reference goes.  The GPU then hashes level by level, all bodies of
// the same length in one launch per level:
//   kind BOTTOM  a full branch whose 16 children are leaves [0x20, rlp(byte)] -> 1 permutation,
//                built from 16 body bytes (the bulk: N/16 nodes);
//   kind HFULL   a full branch whose 16 children are all hashed -> 532-byte message, 4 permutations;
//                children store their raw 32-byte hashes (aligned) into its buffer and the message
//                f9 02 11 | (a0 || H_s) x 16 | 80 is generated word by word at compile-time offsets;
//   kind BRANCH / EXT / LEAF  generic nodes (partial right edge, top of trie, root): assembled
//                byte by byte from children refs, inlined when RLP < 32 bytes (trie/hasher.go:163),
//                the root always hashed (force).
//
// GENERIC plans serve DeriveSha over any DerivableList (tx root core/block_validator.go:70, receipt
// root :92): the same key-only shape, but values are arbitrary byte strings (list.GetRlp(j)), so no
// BOTTOM/HFULL specialisation — every leaf is hashed or inlined by k_derive_leaf at the depth the
// plan records (leaf_depth[j]) and every internal node is a generic BRANCH/EXT.
#pragma once
#include <stdint.h>

#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace gsv {

enum : uint8_t { PK_BOTTOM = 0, PK_HFULL = 1, PK_BRANCH = 2, PK_EXT = 3, PK_LEAF = 4 };
enum : uint8_t { PC_LEAF = 1, PC_NODE = 2 };

struct PNode {
    uint8_t kind;
    uint8_t height;
    uint8_t is_root;
    uint8_t nchild;       // generic: number of child entries
    int32_t msg_off;      // own message buffer offset in the per-body msg arena (-1 for BOTTOM)
    int32_t parent_msg;   // HFULL parent: byte offset in the msg arena of this node's 32-byte hash slot, or -1
    int32_t ref_slot;     // canonical ref slot (generic parents read refs from here)
    uint32_t first_i;     // BOTTOM: body index of child 0; LEAF: body index
    int32_t child_begin;  // generic: first entry in the child array
    uint16_t depth;       // nibbles consumed above this node (EXT: segment start; LEAF: remainder start)
    uint16_t ext_end;     // EXT: segment end (exclusive); EXT segment nibbles are those of key(first_i)
};

struct PChild {
    uint8_t slot;    // branch slot 0..15
    uint8_t type;    // PC_LEAF / PC_NODE
    uint16_t depth;  // leaf: nibble index where its remainder key starts
    uint32_t idx;    // leaf: body index; node: node id
};

constexpr int MSG_STRIDE = 544;  // bytes per message buffer (532 max + padding to the 4th block end);
                                 // an HFULL node's buffer holds its 16 children's raw hashes (512 B)
constexpr int TOP_MAX_HFULL = 1024;  // fused-top eligibility per height (per body)
constexpr int TOP_MAX_GEN = 64;
constexpr int TOP_MAX_H = 24;
constexpr int REF_STRIDE = 48;   // bytes per ref slot: [0] = length, [8..41) = ref bytes

struct TriePlanHost {
    uint32_t N = 0;
    bool generic = false;
    std::vector<uint16_t> leaf_depth;  // generic: nibble index where leaf j's remainder key starts
    std::vector<PNode> nodes;     // sorted by height, BOTTOM first inside height 1
    std::vector<PChild> children;
    // per height h (1..H): [bottom_begin, bottom_end) and [gen_begin, gen_end) node id ranges
    std::vector<int> lvl_bottom_begin, lvl_bottom_end, lvl_hfull_begin, lvl_hfull_end, lvl_gen_begin, lvl_gen_end;
    int height = 0;
    int top_h = 1;  // heights top_h..height run fused in k_chunk_top (one workgroup per body)
    int root = -1;
    int n_msg = 0;    // message buffers per body
    int n_slots = 0;  // ref slots per body
};

struct TriePlan {
    TriePlanHost h;
    PNode* d_nodes = nullptr;
    PChild* d_children = nullptr;
    uint16_t* d_leaf_depth = nullptr;
    size_t bytes = 0;  // host + device footprint
    TriePlan() = default;
    TriePlan(const TriePlan&) = delete;
    TriePlan& operator=(const TriePlan&) = delete;
    ~TriePlan();  // frees the device arrays (also on a failed, partial upload)
};

void build_trie_plan(TriePlanHost& p, uint32_t N, bool generic = false);

// Per-(N, generic) plans, built and uploaded on first use.  Bounded: beyond kMaxBytes the
// least-recently-used plans that no prepared shape holds (use_count == 1: no queued work can read
// them, because a shape drains its work before it is dropped) are freed.
class PlanCache {
  public:
    static constexpr size_t kMaxBytes = (size_t)512 << 20;
    // nullptr when the device upload fails (out of memory)
    std::shared_ptr<TriePlan> get(uint32_t N, bool generic = false);
    size_t bytes() const { return bytes_; }
    size_t size() const { return plans_.size(); }

  private:
    struct Entry {
        std::shared_ptr<TriePlan> plan;
        uint64_t last_use;
    };
    std::mutex mu_;
    std::map<uint64_t, Entry> plans_;
    uint64_t tick_ = 0;
    size_t bytes_ = 0;
};

}  // namespace gsv
