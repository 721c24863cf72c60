// Item -> (row, 16-byte slot) maps for staging [rows][32] 16-bit tiles into LDS rows of an 80-byte
// (five-slot) pitch: the pitch that makes the MFMA fragment reads (ds_read_b128, 16-lane groups over
// 64 banks) conflict-free.  The writes are serviced in smaller groups over 32 banks: a ds_write_b128
// group is 8 lanes (128 B), a ds_write_b64 group 16 lanes.  Consecutive items filling rows r and r + 1
// put slot 5r and slot 5r + 8 (b128) / dwords 20r and 20r + 32 (b64) on the same banks: every write
// instruction took two passes.  Pairing rows r and r + 4 in one group instead (5 * 4 = 20 = 4 mod 8
// slots; 20 * 4 = 80 = 16 mod 32 dwords) spreads a group over distinct banks.  Both maps are bijections
// on a multiple of 8 rows; the global loads use the same map, so only which lane stages which piece
// changes (every piece is still one 16- / 8-byte load from its row).
#pragma once

namespace dsg {

// 16-byte items, 4 per row (bf16 x 8 each): item -> (row, slot 0..3)
__device__ __forceinline__ int p80_row16(int it) { return ((it >> 5) << 3) | ((it >> 3) & 3) | (((it >> 2) & 1) << 2); }
__device__ __forceinline__ int p80_slot16(int it) { return it & 3; }
// 8-byte items, 8 per row (bf16 x 4 each): item -> (row, piece 0..7)
__device__ __forceinline__ int p80_row8(int it) { return ((it >> 6) << 3) | ((it >> 4) & 3) | (((it >> 3) & 1) << 2); }
__device__ __forceinline__ int p80_piece8(int it) { return it & 7; }

}  // namespace dsg
