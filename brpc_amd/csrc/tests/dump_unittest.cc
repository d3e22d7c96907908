// recordio, rpc_dump sampling and byte-for-byte replay (spirit of the
// reference's test/recordio_unittest.cpp and the rpc_dump/rpc_replay pair).
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#include "base/flags.h"
#include "base/recordio.h"
#include "mrpc/proto/echo.pb.h"
#include "mrpc/proto/rpc_dump.pb.h"
#include "rpc/channel.h"
#include "rpc/protocol.h"
#include "rpc/rpc_dump.h"
#include "rpc/serialized_request.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

TEST(RecordIO, write_read_and_resync_after_corruption) {
    const std::string path = "/tmp/mrpc_recordio_" + std::to_string(getpid());
    unlink(path.c_str());
    {
        RecordWriter w(path);
        ASSERT_TRUE(w.ok());
        for (int i = 0; i < 50; ++i) {
            Record r;
            r.MutableMeta("k")->append("meta-" + std::to_string(i));
            if (i % 3 == 0) r.MutableMeta("second")->append(std::string(i, 'x'));
            r.MutablePayload()->append(std::string(i * 37, (char)('a' + i % 26)));
            ASSERT_EQ(w.Write(r), 0);
        }
    }
    // corrupt one byte in the middle of the file
    FILE* f = fopen(path.c_str(), "r+b");
    fseek(f, 0, SEEK_END);
    const long size = ftell(f);
    fseek(f, size / 2, SEEK_SET);
    fputc(0x5a, f);
    fclose(f);
    RecordReader rd(path);
    Record r;
    int n = 0;
    while (rd.ReadNext(&r)) {
        ++n;
        const Buf* k = r.Meta("k");
        ASSERT_TRUE(k != nullptr);
        const int i = atoi(k->to_string().c_str() + 5);
        EXPECT_EQ(r.Payload().size(), (size_t)i * 37);
        EXPECT_EQ(r.Meta("second") != nullptr, i % 3 == 0);
    }
    EXPECT_EQ(rd.last_error(), 0);
    EXPECT_GE(n, 48);  // only the damaged record is lost
    EXPECT_LT(n, 50);
    EXPECT_GT(rd.skipped_bytes(), 0u);
    unlink(path.c_str());
}

TEST(RpcDump, sample_and_replay_byte_for_byte) {
    const std::string dir = "/tmp/mrpc_dump_test_" + std::to_string(getpid());
    SetFlag("rpc_dump_dir", dir);
    SetFlag("rpc_dump", "true");
    Server server;
    EchoServiceImpl echo;
    server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    o.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &o), 0);
    const std::string addr = "127.0.0.1:" + std::to_string(server.listen_port());
    Channel ch;
    ChannelOptions copt;
    ASSERT_EQ(ch.Init(addr.c_str(), &copt), 0);
    example::EchoService_Stub stub(&ch);
    for (int i = 0; i < 20; ++i) {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("dump-" + std::to_string(i));
        cntl.request_attachment().append("att" + std::to_string(i));
        if (i % 2) cntl.set_request_compress_type(COMPRESS_TYPE_SNAPPY);
        stub.Echo(&cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
    }
    SetFlag("rpc_dump", "false");
    FlushRpcDump();
    std::vector<std::string> files = ListRpcDumpFiles(dir);
    ASSERT_GE(files.size(), 1u);
    int nrec = 0;
    const int64_t before = echo.ncalls();
    for (const std::string& fn : files) {
        RecordReader rd(dir + "/" + fn);
        Record r;
        while (rd.ReadNext(&r)) {
            ++nrec;
            RpcDumpMeta meta;
            ASSERT_TRUE(meta.ParseFromBuf(*r.Meta("meta")));
            EXPECT_EQ(meta.service_name(), "example.EchoService");
            EXPECT_EQ(meta.method_name(), "Echo");
            EXPECT_EQ((int)meta.protocol_type(), (int)PROTOCOL_BAIDU_STD);
            // replay exactly those bytes
            Buf payload = r.Payload();
            Buf body;
            payload.cutn(&body, payload.size() - meta.attachment_size());
            Controller cntl;
            SerializedRequest req;
            req.serialized_data() = body;
            cntl.request_attachment() = payload;
            cntl.set_request_compress_type(meta.compress_type());
            example::EchoResponse res;
            ch.CallMethod(example::EchoService::descriptor()->method(0), &cntl, &req, &res, nullptr);
            ASSERT_FALSE(cntl.Failed());
            EXPECT_EQ(res.message().substr(0, 5), "dump-");
            EXPECT_EQ(cntl.response_attachment().to_string().substr(0, 3), "att");
        }
    }
    EXPECT_EQ(nrec, 20);  // below the speed limit every request is sampled
    EXPECT_EQ(echo.ncalls(), before + nrec);
    for (const std::string& fn : files) unlink((dir + "/" + fn).c_str());
    rmdir(dir.c_str());
}

TEST(RpcDump, files_rotate_and_old_ones_are_removed) {
    // 5 requests per file, at most 3 files: 23 sampled requests leave the
    // newest 3 files (the last one partial) and nothing older
    const std::string dir = "/tmp/mrpc_dump_rot_" + std::to_string(getpid());
    SetFlag("rpc_dump_dir", dir);
    SetFlag("rpc_dump_max_requests_in_one_file", "5");
    SetFlag("rpc_dump_max_files", "3");
    SetFlag("rpc_dump", "true");
    Server server;
    EchoServiceImpl echo;
    server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    o.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &o), 0);
    const std::string addr = "127.0.0.1:" + std::to_string(server.listen_port());
    Channel ch;
    ASSERT_EQ(ch.Init(addr.c_str(), nullptr), 0);
    example::EchoService_Stub stub(&ch);
    for (int i = 0; i < 23; ++i) {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("rot-" + std::to_string(i));
        stub.Echo(&cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        if (i % 5 == 4) FlushRpcDump();  // let the collector see the requests in order
    }
    SetFlag("rpc_dump", "false");
    FlushRpcDump();
    std::vector<std::string> files = ListRpcDumpFiles(dir);
    EXPECT_LE(files.size(), 3u);
    ASSERT_GE(files.size(), 1u);
    std::vector<int> seen;
    for (const std::string& fn : files) {
        RecordReader rd(dir + "/" + fn);
        Record r;
        int in_file = 0;
        while (rd.ReadNext(&r)) {
            ++in_file;
            Buf payload = r.Payload();
            example::EchoRequest req;
            ASSERT_TRUE(req.ParseFromBuf(payload));
            seen.push_back(atoi(req.message().c_str() + 4));
        }
        EXPECT_LE(in_file, 5);
    }
    // the newest requests survive, the oldest files were removed
    ASSERT_FALSE(seen.empty());
    EXPECT_EQ(*std::max_element(seen.begin(), seen.end()), 22);
    EXPECT_GT(*std::min_element(seen.begin(), seen.end()), 0);
    EXPECT_LE(seen.size(), 15u);
    SetFlag("rpc_dump_max_requests_in_one_file", "1000");
    SetFlag("rpc_dump_max_files", "32");
    for (const std::string& fn : files) unlink((dir + "/" + fn).c_str());
    rmdir(dir.c_str());
}
