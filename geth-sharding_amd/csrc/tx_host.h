// Host-side transaction decoding for the batch types.Sender path (see tx_host.hip).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../../include/gsv.h"

namespace gsv {

struct TxPrep {
    std::vector<uint8_t> pre;  // RLP sighash preimage for the signer
    uint8_t r32[32], s32[32];
    uint64_t v;     // V as passed to recoverPlain (low 64 bits)
    uint8_t vbig;   // forces GSV_ST_INVALID_SIG (V > 8 bits, or R/S >= 2^256)
    int homestead;  // reject s > n/2
};

// Returns GSV_ST_OK (fills out) or GSV_ST_BAD_RLP / GSV_ST_INVALID_CHAIN_ID / GSV_ST_INVALID_SIG.
int tx_prepare(const uint8_t* rlp, size_t len, const uint8_t* chain_id, size_t chain_id_len,
               int signer_kind, TxPrep& out);

}  // namespace gsv
