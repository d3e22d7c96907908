// More CallId cases (fiber/call_id.h), after the reference's
// test/bthread_id_unittest.cpp (sanity, ranged ids, cancel, join of invalid
// ids, error without a handler): the data pointer round trip, versions of a
// range addressing one object, versions outside the range, cancel only of an
// unlocked id, error on a destroyed id, the default handler, trylock on a
// locked id, join on ids that never existed, and slot reuse keeping old
// versions dead.
#include <atomic>
#include <cerrno>
#include <string>
#include <thread>
#include <vector>

#include "fiber/call_id.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::fiber;

namespace {

struct Box {
    int value = 0;
    std::atomic<int> errors{0};
    int last_code = 0;
    std::string last_text;
};

int box_on_error(CallId id, void* data, int code, const std::string& text) {
    Box* b = static_cast<Box*>(data);
    b->errors.fetch_add(1);
    b->last_code = code;
    b->last_text = text;
    return call_id_unlock(id);
}

int destroy_on_error(CallId id, void* data, int code, const std::string& text) {
    Box* b = static_cast<Box*>(data);
    b->errors.fetch_add(1);
    b->last_code = code;
    b->last_text = text;
    return call_id_unlock_and_destroy(id);
}

}  // namespace

TEST(CallIdMore, lock_hands_back_the_data_pointer) {
    Box box;
    CallId id;
    ASSERT_EQ(call_id_create(&id, &box, box_on_error), 0);
    EXPECT_TRUE(id != INVALID_CALL_ID);
    EXPECT_TRUE(call_id_exists(id));
    void* data = nullptr;
    ASSERT_EQ(call_id_lock(id, &data), 0);
    EXPECT_TRUE(data == &box);
    static_cast<Box*>(data)->value = 42;
    ASSERT_EQ(call_id_unlock(id), 0);
    ASSERT_EQ(call_id_lock(id, nullptr), 0);  // data pointer is optional
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
    EXPECT_FALSE(call_id_exists(id));
    EXPECT_EQ(box.value, 42);
}

TEST(CallIdMore, every_version_of_a_range_names_the_same_id) {
    Box box;
    CallId base;
    ASSERT_EQ(call_id_create_ranged(&base, &box, box_on_error, 4), 0);
    for (int v = 0; v < 4; ++v) {
        CallId idv = call_id_with_version(base, v);
        EXPECT_EQ(call_id_version(idv), call_id_version(base) + (uint32_t)v);
        void* data = nullptr;
        ASSERT_EQ(call_id_lock(idv, &data), 0);
        EXPECT_TRUE(data == &box);
        ASSERT_EQ(call_id_unlock(idv), 0);
    }
    // one past the range is not this id
    EXPECT_EQ(call_id_lock(call_id_with_version(base, 4), nullptr), EINVAL);
    ASSERT_EQ(call_id_lock(base, nullptr), 0);
    ASSERT_EQ(call_id_unlock_and_destroy(base), 0);
    for (int v = 0; v < 4; ++v) EXPECT_FALSE(call_id_exists(call_id_with_version(base, v)));
}

TEST(CallIdMore, cancel_destroys_an_unlocked_id_only) {
    Box box;
    CallId id;
    ASSERT_EQ(call_id_create(&id, &box, box_on_error), 0);
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    EXPECT_NE(call_id_cancel(id), 0);  // locked: refused
    ASSERT_EQ(call_id_unlock(id), 0);
    EXPECT_EQ(call_id_cancel(id), 0);
    EXPECT_FALSE(call_id_exists(id));
    EXPECT_EQ(call_id_cancel(id), EINVAL);
}

TEST(CallIdMore, error_runs_the_handler_with_code_and_text) {
    Box box;
    CallId id;
    ASSERT_EQ(call_id_create(&id, &box, box_on_error), 0);
    ASSERT_EQ(call_id_error(id, ETIMEDOUT, "too slow"), 0);
    EXPECT_EQ(box.errors.load(), 1);
    EXPECT_EQ(box.last_code, ETIMEDOUT);
    EXPECT_EQ(box.last_text, std::string("too slow"));
    EXPECT_TRUE(call_id_exists(id));  // the handler only unlocked it
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
}

TEST(CallIdMore, error_on_a_destroyed_id_is_refused) {
    Box box;
    CallId id;
    ASSERT_EQ(call_id_create(&id, &box, destroy_on_error), 0);
    ASSERT_EQ(call_id_error(id, ECANCELED), 0);
    EXPECT_FALSE(call_id_exists(id));
    EXPECT_EQ(call_id_error(id, ECANCELED), EINVAL);
    EXPECT_EQ(box.errors.load(), 1);
}

TEST(CallIdMore, without_a_handler_error_destroys_the_id) {
    CallId id;
    ASSERT_EQ(call_id_create(&id, nullptr, nullptr), 0);
    EXPECT_EQ(call_id_error(id, EINTR), 0);
    EXPECT_FALSE(call_id_exists(id));
    EXPECT_EQ(call_id_join(id), 0);
}

TEST(CallIdMore, trylock_on_a_locked_id_is_busy) {
    Box box;
    CallId id;
    ASSERT_EQ(call_id_create(&id, &box, box_on_error), 0);
    ASSERT_EQ(call_id_trylock(id, nullptr), 0);
    EXPECT_EQ(call_id_trylock(id, nullptr), EBUSY);
    std::atomic<int> rc{-1};
    std::thread t([&] { rc = call_id_trylock(id, nullptr); });
    t.join();
    EXPECT_EQ(rc.load(), EBUSY);
    ASSERT_EQ(call_id_unlock(id), 0);
    ASSERT_EQ(call_id_trylock(id, nullptr), 0);
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
    EXPECT_EQ(call_id_trylock(id, nullptr), EINVAL);
}

TEST(CallIdMore, join_of_ids_that_never_existed_does_not_block) {
    EXPECT_EQ(call_id_join(INVALID_CALL_ID), 0);
    CallId bogus{0x123456789abcdefull};
    EXPECT_EQ(call_id_join(bogus), EINVAL);  // a slot never allocated
    EXPECT_FALSE(call_id_exists(bogus));
    EXPECT_EQ(call_id_lock(bogus, nullptr), EINVAL);
    EXPECT_EQ(call_id_unlock(bogus), EINVAL);
}

TEST(CallIdMore, a_recycled_slot_gets_new_versions) {
    std::vector<CallId> old;
    for (int i = 0; i < 64; ++i) {
        CallId id;
        ASSERT_EQ(call_id_create_ranged(&id, nullptr, nullptr, 3), 0);
        old.push_back(id);
        ASSERT_EQ(call_id_cancel(id), 0);
    }
    for (int i = 0; i < 64; ++i) {
        CallId id;
        ASSERT_EQ(call_id_create(&id, nullptr, nullptr), 0);
        for (const CallId& o : old) {
            for (int v = 0; v < 3; ++v) EXPECT_TRUE(call_id_with_version(o, v) != id);
        }
        ASSERT_EQ(call_id_cancel(id), 0);
    }
    for (const CallId& o : old) EXPECT_FALSE(call_id_exists(o));
}

TEST(CallIdMore, joiners_on_fibers_and_threads_all_wake) {
    CallId id;
    ASSERT_EQ(call_id_create(&id, nullptr, nullptr), 0);
    std::atomic<int> woke{0};
    CountdownEvent fibers(3);
    for (int i = 0; i < 3; ++i) {
        start([&] {
            call_id_join(id);
            woke.fetch_add(1);
            fibers.signal();
        });
    }
    std::vector<std::thread> ts;
    for (int i = 0; i < 3; ++i) {
        ts.emplace_back([&] {
            call_id_join(id);
            woke.fetch_add(1);
        });
    }
    usleep(20000);
    EXPECT_EQ(woke.load(), 0);
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
    for (auto& t : ts) t.join();
    fibers.wait();
    EXPECT_EQ(woke.load(), 6);
}

TEST(CallIdMore, unlock_of_an_unlocked_id_is_refused) {
    CallId id;
    ASSERT_EQ(call_id_create(&id, nullptr, nullptr), 0);
    EXPECT_NE(call_id_unlock(id), 0);
    EXPECT_NE(call_id_unlock_and_destroy(id), 0);
    EXPECT_TRUE(call_id_exists(id));
    ASSERT_EQ(call_id_cancel(id), 0);
}
