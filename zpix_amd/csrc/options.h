// Process-wide test switches (zpx_debug_option, include/zpix_amd.h): which
// kernel or transport a path takes where two produce the same result.  Not
// read from the environment: the shipped library takes one path unless a
// test says so.
#pragma once

namespace zpx {

enum class Opt { JpegStrip, JpegSparse, PngPair, QoiSegment, PngDeviceSlab, PngEpochCycle, ShardRcclSelf, BatchLookahead, InflatePair, BatchMakespan, BatchSlotCache, Count };
int opt(Opt o);

} // namespace zpx
