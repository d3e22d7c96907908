// Host half of the device-payload codec (gpu/device_codec.h): the block
// layout, the block-table validation a receiver runs before launching
// anything (a bad table must never reach the decoder), and the wire form of
// the descriptor's block table. The device half runs in
// tests/test_gpu_device_codec.py on the GPU box.
#include <string>
#include <vector>

#include "base/flags.h"
#include "gpu/codec_batch.h"
#include "gpu/device_codec.h"
#include "gpu/kernels.h"
#include "mrpc/proto/device_payload.pb.h"
#include "policy/device_payload.h"
#include "tests/test.h"

DECLARE_int32(device_payload_block_kb);

using namespace mrpc;

namespace {

gpu::DeviceSnappyBlocks job(const std::vector<uint32_t>& clen, uint64_t len, uint64_t region_len,
                            uint32_t ulen = 4096, uint32_t stride = 4816) {
    static char region[1];
    static char dst[1];
    gpu::DeviceSnappyBlocks j;
    j.region = region;  // never dereferenced: every case here is refused
    j.region_len = region_len;
    j.lay.block_ulen = ulen;
    j.lay.stride = stride;
    j.lay.nblocks = (uint32_t)clen.size();
    j.clen = clen.data();
    j.dst = dst;
    j.len = len;
    return j;
}

int decode_code(const gpu::DeviceSnappyBlocks& j) {
    int err = -1;
    DevicePayloadIndex idx;
    const int rc = gpu::DeviceSnappyDecode(&j, 1, &err, &idx, 0);
    return rc != 0 ? -100 : err;
}

}  // namespace

TEST(DeviceCodec, layout_covers_the_payload_with_worst_case_strides) {
    const int saved = FLAGS_device_payload_block_kb;
    FLAGS_device_payload_block_kb = 4;
    const gpu::DeviceSnappyLayout l = gpu::DeviceSnappyLayoutFor(65536);
    EXPECT_EQ(l.block_ulen, 4096u);
    EXPECT_EQ(l.nblocks, 16u);
    EXPECT_GE(l.stride, (uint32_t)gpu::SnappyMaxCompressedLength(4096));
    EXPECT_EQ(l.stride % 16, 0u);
    EXPECT_EQ(l.region(), (uint64_t)l.stride * 16);
    EXPECT_EQ(gpu::DeviceSnappyLayoutFor(1).nblocks, 1u);
    EXPECT_EQ(gpu::DeviceSnappyLayoutFor(4097).nblocks, 2u);
    EXPECT_EQ(gpu::DeviceSnappyLayoutFor(1 << 20).nblocks, 256u);
    FLAGS_device_payload_block_kb = saved;
    EXPECT_EQ(gpu::DeviceSnappyLayoutFor(65536).block_ulen, 2048u);  // the default
}

TEST(DeviceCodec, layout_follows_the_block_flag_within_bounds) {
    const int saved = FLAGS_device_payload_block_kb;
    FLAGS_device_payload_block_kb = 16;
    EXPECT_EQ(gpu::DeviceSnappyLayoutFor(65536).block_ulen, 16384u);
    FLAGS_device_payload_block_kb = 1000;  // clamped to one snappy block
    EXPECT_EQ(gpu::DeviceSnappyLayoutFor(65536).block_ulen, gpu::kSnappyMaxBlock);
    FLAGS_device_payload_block_kb = 0;
    EXPECT_EQ(gpu::DeviceSnappyLayoutFor(65536).block_ulen, 1024u);
    FLAGS_device_payload_block_kb = saved;
}

TEST(DeviceCodec, bad_block_tables_are_refused_before_any_launch) {
    const uint64_t len = 10000;  // 3 blocks of 4096, 4096, 1808
    const uint64_t region = 3 * 4816;
    const int64_t before = gpu::GetDeviceCodecStats().bad_tables;
    // too few / too many blocks for the payload
    EXPECT_EQ(decode_code(job({100, 100}, len, region)), 1);
    EXPECT_EQ(decode_code(job({100, 100, 100, 100}, len, region)), 1);
    // a block longer than its slot, or one past the region
    EXPECT_EQ(decode_code(job({4817, 100, 100}, len, region)), 1);
    EXPECT_EQ(decode_code(job({100, 100, 100}, len, 2 * 4816 + 99)), 1);
    // a block holding no more than its varint header (4096 needs 2 bytes)
    EXPECT_EQ(decode_code(job({2, 100, 100}, len, region)), 1);
    EXPECT_EQ(decode_code(job({100, 100, 0}, len, region)), 1);
    // nonsense geometry
    EXPECT_EQ(decode_code(job({100, 100, 100}, len, region, 0)), 1);
    EXPECT_EQ(decode_code(job({100, 100, 100}, len, region, 4096, 0)), 1);
    EXPECT_EQ(decode_code(job({100}, 70000, region, 70000, 90000)), 1);  // block above kSnappyMaxBlock
    EXPECT_EQ(decode_code(job({}, len, region)), 1);
    EXPECT_EQ(decode_code(job({100}, 0, region)), 1);
    EXPECT_EQ(gpu::GetDeviceCodecStats().bad_tables - before, 11);
}

TEST(DeviceCodec, mixed_jobs_report_per_job_codes) {
    // every job bad: nothing is launched, each gets its own code
    std::vector<uint32_t> a{100, 100}, b{5000};
    gpu::DeviceSnappyBlocks jobs[2] = {job(a, 10000, 3 * 4816), job(b, 100, 4816)};
    int err[2] = {-1, -1};
    DevicePayloadIndex idx[2];
    EXPECT_EQ(gpu::DeviceSnappyDecode(jobs, 2, err, idx, 0), 0);
    EXPECT_EQ(err[0], 1);
    EXPECT_EQ(err[1], 1);
    EXPECT_EQ(idx[0].nfields, -1);
}

TEST(DeviceCodec, descriptor_block_table_round_trips_on_the_wire) {
    policy::DevicePayload d;
    d.set_ring_offset(1 << 20);
    d.set_length(65536);
    d.set_lent_length(16 * 4816);
    d.set_compress_type(1);
    d.set_block_stride(4816);
    d.set_block_ulen(4096);
    for (uint32_t i = 0; i < 16; ++i) d.add_block_clen(1000 + 37 * i);
    d.set_pb_scan(true);
    std::string wire;
    ASSERT_TRUE(d.SerializeToString(&wire));
    policy::DevicePayload back;
    ASSERT_TRUE(back.ParseFromString(wire));
    EXPECT_EQ(back.length(), 65536);
    EXPECT_EQ(back.lent_length(), 16 * 4816);
    EXPECT_EQ(back.compress_type(), 1);
    EXPECT_EQ(back.block_stride(), 4816u);
    EXPECT_EQ(back.block_ulen(), 4096u);
    ASSERT_EQ(back.block_clen_size(), 16);
    for (int i = 0; i < 16; ++i) EXPECT_EQ(back.block_clen(i), 1000u + 37u * (uint32_t)i);
    EXPECT_TRUE(back.pb_scan());
    // a descriptor of an older sender (no table) reads as an uncompressed lend
    policy::DevicePayload old;
    old.set_ring_offset(4096);
    old.set_length(100);
    std::string w2;
    ASSERT_TRUE(old.SerializeToString(&w2));
    policy::DevicePayload b2;
    ASSERT_TRUE(b2.ParseFromString(w2));
    EXPECT_EQ(b2.compress_type(), 0);
    EXPECT_EQ(b2.block_clen_size(), 0);
    EXPECT_FALSE(b2.pb_scan());
}

TEST(DeviceCodec, payload_field_lookup_reads_length_delimited_entries) {
    DevicePayloadIndex idx;
    idx.nfields = 3;
    idx.fields = {(1u << 3) | 0, 42,                                  // varint field 1
                  (2u << 3) | 2, (7ull << 32) | 1000,                 // bytes field 2
                  (2u << 3) | 2, (2000ull << 32) | 5};                // a repeated second entry
    uint64_t off = 0, len = 0;
    EXPECT_FALSE(gpu::DevicePayloadField(idx, 1, &off, &len));  // not length-delimited
    ASSERT_TRUE(gpu::DevicePayloadField(idx, 2, &off, &len));
    EXPECT_EQ(off, 7u);
    EXPECT_EQ(len, 1000u);
    EXPECT_FALSE(gpu::DevicePayloadField(idx, 3, &off, &len));
    idx.nfields = -1;  // not scanned
    EXPECT_FALSE(gpu::DevicePayloadField(idx, 2, &off, &len));
    idx.nfields = 5;  // more than the table holds: bounded by the table
    EXPECT_TRUE(gpu::DevicePayloadField(idx, 2, &off, &len));
}

TEST(DeviceCodec, packed_runs_with_bad_arguments_are_refused_before_any_launch) {
    static char buf[16];
    gpu::DevicePackedRun runs[4];
    runs[0].src = nullptr;  // no source
    runs[0].dst = buf;
    runs[0].len = 4;
    runs[1].src = buf;  // no destination
    runs[1].len = 4;
    runs[2].src = buf;  // unknown kind
    runs[2].dst = buf;
    runs[2].len = 4;
    runs[2].kind = 99;
    runs[3].src = buf;  // empty: nothing to decode, not an error
    runs[3].dst = buf;
    runs[3].len = 0;
    EXPECT_EQ(gpu::DeviceDecodePackedRuns(runs, 4, 0), 0);
    EXPECT_EQ(runs[0].err, 2);
    EXPECT_EQ(runs[1].err, 2);
    EXPECT_EQ(runs[2].err, 2);
    EXPECT_EQ(runs[3].err, 0);
    EXPECT_EQ(runs[3].count, 0u);
    EXPECT_EQ(gpu::DeviceDecodePackedRuns(runs, 0, 0), 0);
}

TEST(DeviceCodec, pooled_request_reset_matches_a_fresh_one) {
    // the device codec reuses CodecRequests from a pool: Reset() must leave
    // every job list and result empty and every limit at its default, or a
    // pooled request would carry jobs of the previous RPC into the next batch
    gpu::CodecRequest r;
    const gpu::CodecRequest fresh;
    r.runs.resize(2);
    r.h2d.resize(3);
    r.comp.resize(4);
    r.decomp.resize(5);
    r.comp_max_ulen = 77;
    r.decomp_max_ulen = 88;
    r.streams.resize(1);
    r.stream_piece_limit = 123;
    r.pieces.resize(6);
    r.pieces_max_ulen = 99;
    r.scans.resize(2);
    r.scan_piece_first.resize(2);
    r.scan_piece_count.resize(2);
    r.d2h.resize(1);
    r.dec_runs.resize(3);
    r.comp_len.resize(4);
    r.decomp_len.resize(5);
    r.comp_err.resize(4);
    r.decomp_err.resize(5);
    r.stream_err.resize(1);
    r.piece_err.resize(6);
    r.run_err.resize(2);
    r.dec_counts.resize(3);
    r.dec_err.resize(3);
    r.scan_fields.resize(8);
    r.scan_nfields.resize(2);
    const size_t cap = r.pieces.capacity();
    r.Reset();
    EXPECT_TRUE(r.runs.empty() && r.h2d.empty() && r.comp.empty() && r.decomp.empty() && r.streams.empty());
    EXPECT_TRUE(r.pieces.empty() && r.scans.empty() && r.scan_piece_first.empty() && r.scan_piece_count.empty());
    EXPECT_TRUE(r.d2h.empty() && r.dec_runs.empty() && r.comp_len.empty() && r.decomp_len.empty());
    EXPECT_TRUE(r.comp_err.empty() && r.decomp_err.empty() && r.stream_err.empty() && r.piece_err.empty());
    EXPECT_TRUE(r.run_err.empty() && r.dec_counts.empty() && r.dec_err.empty() && r.scan_fields.empty());
    EXPECT_TRUE(r.scan_nfields.empty());
    EXPECT_EQ(r.comp_max_ulen, fresh.comp_max_ulen);
    EXPECT_EQ(r.decomp_max_ulen, fresh.decomp_max_ulen);
    EXPECT_EQ(r.stream_piece_limit, fresh.stream_piece_limit);
    EXPECT_EQ(r.pieces_max_ulen, fresh.pieces_max_ulen);
    EXPECT_EQ(r.pieces.capacity(), cap);  // capacity kept: no allocation on the next use
    // 22 lists and 4 limits (x86-64 layout, with the padding after the two
    // lone limits): a member added later changes the size, and this test
    // (and Reset()) must learn about it
    EXPECT_EQ(sizeof(gpu::CodecRequest), 22 * sizeof(std::vector<int>) + 4 * sizeof(uint32_t) + 8);
}
