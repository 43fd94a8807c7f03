// render_core_flags.h -- constants shared by the host layout compiler and the kernel.
#pragma once
#define ORT_INTERNAL_FLAG_HOST 0x80000000u
#define ORT_LEAFKIDS_FLAG_HOST 0x40000000u  // internal node whose existing children are all leaves
#define ORT_COMPACT_MAX_DEPTH_HOST 10
#define ORT_LEAFMASK_SHIFT_HOST 8           // internal node: bits 8-15 = its existing leaf children
