// SocketMap: one shared client connection per (endpoint, signature)
// (spirit of the reference's test/brpc_socket_map_unittest.cpp):
// reference counting, signatures that separate connections, replacement of
// a failed socket, concurrent users, and Channels that share a connection.
#include <atomic>
#include <set>
#include <thread>
#include <vector>

#include "base/endpoint.h"
#include "mrpc/proto/echo.pb.h"
#include "net/socket.h"
#include "net/socket_map.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {
SocketMapKey key_of(int port, const std::string& sig = "") {
    SocketMapKey k;
    str2endpoint("127.0.0.1", port, &k.peer);
    k.signature = sig;
    return k;
}
}  // namespace

TEST(SocketMapUnit, refcounted_entries_share_one_socket) {
    const size_t before = SocketMapSize();
    const SocketMapKey k = key_of(1);  // never connected: sockets connect lazily
    SocketId a = INVALID_SOCKET_ID, b = INVALID_SOCKET_ID, found = INVALID_SOCKET_ID;
    ASSERT_EQ(SocketMapInsert(k, &a), 0);
    ASSERT_EQ(SocketMapInsert(k, &b), 0);
    EXPECT_EQ(a, b);
    EXPECT_EQ(SocketMapSize(), before + 1);
    ASSERT_EQ(SocketMapFind(k, &found), 0);
    EXPECT_EQ(found, a);
    SocketMapRemove(k);  // one user left
    EXPECT_EQ(SocketMapFind(k, &found), 0);
    SocketMapRemove(k);  // last user: entry and socket go
    EXPECT_NE(SocketMapFind(k, &found), 0);
    EXPECT_EQ(SocketMapSize(), before);
    SocketMapRemove(k);  // removing an absent key is harmless
    EXPECT_EQ(SocketMapSize(), before);
}

TEST(SocketMapUnit, signatures_and_endpoints_separate_connections) {
    const size_t before = SocketMapSize();
    SocketId plain, auth, other;
    ASSERT_EQ(SocketMapInsert(key_of(2), &plain), 0);
    ASSERT_EQ(SocketMapInsert(key_of(2, "|auth:x"), &auth), 0);
    ASSERT_EQ(SocketMapInsert(key_of(3), &other), 0);
    EXPECT_NE(plain, auth);
    EXPECT_NE(plain, other);
    EXPECT_EQ(SocketMapSize(), before + 3);
    SocketMapRemove(key_of(2));
    SocketMapRemove(key_of(2, "|auth:x"));
    SocketMapRemove(key_of(3));
    EXPECT_EQ(SocketMapSize(), before);
}

TEST(SocketMapUnit, failed_socket_is_replaced_on_insert) {
    const SocketMapKey k = key_of(4);
    SocketId first, second;
    ASSERT_EQ(SocketMapInsert(k, &first), 0);
    // a socket that failed but is still referenced keeps its entry
    // (health checking may revive it): AddressFailedAsWell still sees it
    SocketUniquePtr p;
    ASSERT_EQ(Socket::Address(first, &p), 0);
    p->SetFailed();
    p.reset();
    ASSERT_EQ(SocketMapInsert(k, &second), 0);
    SocketMapRemove(k);
    SocketMapRemove(k);
    SocketId gone;
    EXPECT_NE(SocketMapFind(k, &gone), 0);
}

TEST(SocketMapUnit, concurrent_insert_remove_balances) {
    const size_t before = SocketMapSize();
    std::vector<std::thread> ths;
    std::atomic<int> errors{0};
    std::vector<std::set<SocketId>> seen(8);
    for (int t = 0; t < 8; ++t) {
        ths.emplace_back([t, &errors, &seen] {
            for (int i = 0; i < 500; ++i) {
                const SocketMapKey k = key_of(100 + (i % 4));
                SocketId id;
                if (SocketMapInsert(k, &id) != 0) {
                    errors.fetch_add(1);
                    continue;
                }
                seen[t].insert(id);
                SocketMapRemove(k);
            }
        });
    }
    for (auto& th : ths) th.join();
    EXPECT_EQ(errors.load(), 0);
    EXPECT_EQ(SocketMapSize(), before);  // every insert was matched by a remove
}

TEST(SocketMapUnit, channels_to_one_server_share_the_connection) {
    Server server;
    EchoServiceImpl svc;
    ASSERT_EQ(server.AddService(&svc, SERVER_DOESNT_OWN_SERVICE), 0);
    ServerOptions so;
    so.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &so), 0);
    const std::string addr = "127.0.0.1:" + std::to_string(server.listen_port());
    const size_t before = SocketMapSize();
    {
        Channel a, b;
        ASSERT_EQ(a.Init(addr.c_str(), nullptr), 0);
        ASSERT_EQ(b.Init(addr.c_str(), nullptr), 0);
        EXPECT_EQ(SocketMapSize(), before + 1);  // one shared single connection
        for (Channel* ch : {&a, &b}) {
            example::EchoService_Stub stub(ch);
            Controller cntl;
            example::EchoRequest req;
            example::EchoResponse res;
            req.set_message("shared");
            stub.Echo(&cntl, &req, &res, nullptr);
            ASSERT_FALSE(cntl.Failed());
            EXPECT_EQ(res.message(), "shared");
        }
    }
    EXPECT_EQ(SocketMapSize(), before);  // released with the last channel
    server.Stop(0);
    server.Join();
}
