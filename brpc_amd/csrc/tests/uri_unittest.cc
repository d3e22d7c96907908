// URI depth (http/http_header.h URI), in the spirit of the reference's
// test/brpc_uri_unittest.cpp: every component with and without scheme,
// user info and host, surrounding and embedded spaces, empty and repeated
// query segments, lazy query parsing with order-preserving re-serialization,
// h2 :path round trips and IPv6 hosts.
#include <string>

#include "http/http_header.h"
#include "tests/test.h"

using namespace mrpc;

TEST(UriDepth, everything) {
    URI u;
    ASSERT_EQ(u.SetHttpURL(" foobar://user:passwd@www.example.com:80/s?wd=uri#frag  "), 0);
    EXPECT_EQ(u.scheme(), "foobar");
    EXPECT_EQ(u.port(), 80);
    EXPECT_EQ(u.host(), "www.example.com");
    EXPECT_EQ(u.path(), "/s");
    EXPECT_EQ(u.user_info(), "user:passwd");
    EXPECT_EQ(u.fragment(), "frag");
    ASSERT_TRUE(u.GetQuery("wd") != nullptr);
    EXPECT_EQ(*u.GetQuery("wd"), "uri");
    EXPECT_TRUE(u.GetQuery("nonkey") == nullptr);
}

TEST(UriDepth, only_host) {
    URI u;
    ASSERT_EQ(u.SetHttpURL("  foo1://www.h1.com?wd=uri2&nonkey=22 "), 0);
    EXPECT_EQ(u.scheme(), "foo1");
    EXPECT_EQ(u.port(), -1);
    EXPECT_EQ(u.host(), "www.h1.com");
    EXPECT_EQ(u.path(), "");
    EXPECT_EQ(u.QueryCount(), 2u);
    EXPECT_EQ(*u.GetQuery("nonkey"), "22");
    ASSERT_EQ(u.SetHttpURL("foo2://www.h2.com:1234?wd=uri2&nonkey=22 "), 0);
    EXPECT_EQ(u.port(), 1234);
    EXPECT_EQ(u.host(), "www.h2.com");
    EXPECT_EQ(u.path(), "");
    ASSERT_EQ(u.SetHttpURL(" www.h3.com:4321 "), 0);
    EXPECT_EQ(u.scheme(), "");
    EXPECT_EQ(u.port(), 4321);
    EXPECT_EQ(u.host(), "www.h3.com");
    EXPECT_EQ(u.QueryCount(), 0u);
    ASSERT_EQ(u.SetHttpURL(" www.h4.com "), 0);
    EXPECT_EQ(u.port(), -1);
    EXPECT_EQ(u.host(), "www.h4.com");
    EXPECT_EQ(u.path(), "");
}

TEST(UriDepth, no_scheme_with_and_without_user_info) {
    URI u;
    ASSERT_EQ(u.SetHttpURL(" user:passwd2@www.h1.com/s?wd=uri2&nonkey=22#frag "), 0);
    EXPECT_EQ(u.scheme(), "");
    EXPECT_EQ(u.host(), "www.h1.com");
    EXPECT_EQ(u.path(), "/s");
    EXPECT_EQ(u.user_info(), "user:passwd2");
    EXPECT_EQ(u.fragment(), "frag");
    EXPECT_EQ(*u.GetQuery("wd"), "uri2");
    ASSERT_EQ(u.SetHttpURL(" www.h2.com/s?wd=uri2&nonkey=22#frag "), 0);
    EXPECT_EQ(u.user_info(), "");
    EXPECT_EQ(u.host(), "www.h2.com");
    EXPECT_EQ(u.path(), "/s");
}

TEST(UriDepth, no_host_and_set_path) {
    URI u;
    ASSERT_EQ(u.SetHttpURL(" /sb?wd=uri3#frag2 "), 0);
    EXPECT_EQ(u.host(), "");
    EXPECT_EQ(u.path(), "/sb");
    EXPECT_EQ(u.fragment(), "frag2");
    EXPECT_EQ(*u.GetQuery("wd"), "uri3");
    u.set_path("/x/y/z/");
    EXPECT_EQ(u.path(), "/x/y/z/");
    EXPECT_EQ(*u.GetQuery("wd"), "uri3");  // the rest is untouched
    EXPECT_EQ(u.fragment(), "frag2");
}

TEST(UriDepth, empty_segments_and_keys) {
    URI u;
    u.SetH2Path("/p?&key1=value1&&key3=value3");
    EXPECT_EQ(*u.GetQuery("key1"), "value1");
    EXPECT_EQ(*u.GetQuery("key3"), "value3");
    EXPECT_TRUE(u.GetQuery("key2") == nullptr);
    u.SetH2Path("/p?key1=&&key2&&=&key3=value3");
    ASSERT_TRUE(u.GetQuery("key1") != nullptr);
    EXPECT_EQ(*u.GetQuery("key1"), "");
    ASSERT_TRUE(u.GetQuery("key2") != nullptr);
    EXPECT_EQ(*u.GetQuery("key2"), "");
    EXPECT_EQ(*u.GetQuery("key3"), "value3");
    EXPECT_EQ(u.QueryCount(), 3u);  // the lone "=" has no key
    u.SetH2Path("/p?key1");
    ASSERT_TRUE(u.GetQuery("key1") != nullptr);
    EXPECT_EQ(*u.GetQuery("key1"), "");
}

TEST(UriDepth, set_and_remove_query) {
    URI u;
    u.SetH2Path("/p?key1=&&key2&&=&key3=value3");
    u.SetQuery("key3", "value4");
    EXPECT_EQ(*u.GetQuery("key3"), "value4");
    u.SetQuery("key2", "value2");
    EXPECT_EQ(*u.GetQuery("key2"), "value2");
    u.SetQuery("key9", "new");
    EXPECT_EQ(u.QueryCount(), 4u);
    EXPECT_EQ(u.RemoveQuery("key1"), 1u);
    EXPECT_EQ(u.RemoveQuery("key1"), 0u);
    EXPECT_EQ(u.QueryCount(), 3u);
    EXPECT_EQ(u.query(), "key2=value2&key3=value4&key9=new");  // original order kept
}

TEST(UriDepth, h2_path_round_trips_untouched_queries) {
    URI u;
    const std::string r1 = "/dir?key1=&&key2&&=&key3=value3";
    u.SetH2Path(r1);
    EXPECT_EQ(u.path(), "/dir");
    EXPECT_EQ(u.QueryCount(), 3u);
    std::string out;
    u.GenerateH2Path(&out);
    EXPECT_EQ(out, r1);  // byte for byte while nothing changed
    u.SetQuery("key3", "value3.3");
    EXPECT_EQ(u.RemoveQuery("key1"), 1u);
    EXPECT_EQ(u.query(), "key2&key3=value3.3");
    u.GenerateH2Path(&out);
    EXPECT_EQ(out, "/dir?key2&key3=value3.3");
    const std::string r2 = "/dir2?key1=&&key2&&=&key3=value3#frag2";
    u.SetH2Path(r2);
    EXPECT_EQ(u.fragment(), "frag2");
    u.GenerateH2Path(&out);
    EXPECT_EQ(out, r2);
    u.SetH2Path("/dir3#frag3");
    u.GenerateH2Path(&out);
    EXPECT_EQ(out, "/dir3#frag3");
    u.SetH2Path("dir?a=1");
    EXPECT_EQ(u.path(), "dir");
    EXPECT_EQ(*u.GetQuery("a"), "1");
}

TEST(UriDepth, empty_host) {
    URI u;
    ASSERT_EQ(u.SetHttpURL("http://"), 0);
    EXPECT_EQ(u.host(), "");
    EXPECT_EQ(u.path(), "");
}

TEST(UriDepth, spaces_inside_are_refused_where_they_are) {
    URI u;
    const char* url_bad[] = {"foo bar://user:passwd@www.h.com:80/s?wd=uri#frag",
                             "foobar://us er:passwd@www.h.com:80/s?wd=uri#frag",
                             "foobar://user:pass wd@www.h.com:80/s?wd=uri#frag",
                             "foobar://user:passwd@www. h.com:80/s?wd=uri#frag"};
    for (const char* x : url_bad) {
        EXPECT_EQ(u.SetHttpURL(x), -1);
        EXPECT_EQ(u.status(), "Invalid space in url");
    }
    EXPECT_EQ(u.SetHttpURL("foobar://user:passwd@www.h.com:80/ s?wd=uri#frag"), -1);
    EXPECT_EQ(u.status(), "Invalid space in path");
    EXPECT_EQ(u.SetHttpURL("foobar://user:passwd@www.h.com:80/s ?wd=uri#frag"), -1);
    EXPECT_EQ(u.status(), "Invalid space in path");
    EXPECT_EQ(u.SetHttpURL("foobar://user:passwd@www.h.com:80/s? wd=uri#frag"), -1);
    EXPECT_EQ(u.status(), "Invalid space in query");
    EXPECT_EQ(u.SetHttpURL("foobar://user:passwd@www.h.com:80/s?wd=uri #frag"), -1);
    EXPECT_EQ(u.status(), "Invalid space in query");
    EXPECT_EQ(u.SetHttpURL("foobar://user:passwd@www.h.com:80/s?wd=uri# frag"), -1);
    EXPECT_EQ(u.status(), "Invalid space in fragment");
    EXPECT_EQ(u.SetHttpURL("/a\x01" "b"), -1);  // control characters too
}

TEST(UriDepth, ports_are_checked) {
    URI u;
    EXPECT_EQ(u.SetHttpURL("http://h:65535/"), 0);
    EXPECT_EQ(u.port(), 65535);
    EXPECT_EQ(u.SetHttpURL("http://h:65536/"), -1);
    EXPECT_EQ(u.SetHttpURL("http://h:8o/"), -1);
    EXPECT_EQ(u.status(), "Invalid port");
    EXPECT_EQ(u.SetHttpURL("http://h:/"), 0);  // an empty port is no port
    EXPECT_EQ(u.port(), -1);
}

TEST(UriDepth, ipv6_hosts) {
    URI u;
    ASSERT_EQ(u.SetHttpURL("http://[::1]:8080/p?x=1"), 0);
    EXPECT_EQ(u.host(), "::1");
    EXPECT_EQ(u.port(), 8080);
    EXPECT_EQ(u.path(), "/p");
    EXPECT_EQ(u.to_string(), "http://[::1]:8080/p?x=1");
    ASSERT_EQ(u.SetHttpURL("http://[fe80::1%25eth0]/"), 0);
    EXPECT_EQ(u.host(), "fe80::1%25eth0");
    EXPECT_EQ(u.port(), -1);
    EXPECT_EQ(u.SetHttpURL("http://[::1/"), -1);
    EXPECT_EQ(u.SetHttpURL("http://[::1]x/"), -1);
}

TEST(UriDepth, print_and_copy) {
    URI u;
    ASSERT_EQ(u.SetHttpURL("http://user@h.com:81/a/b?k=v%20w#f"), 0);
    EXPECT_EQ(*u.GetQuery("k"), "v w");
    EXPECT_EQ(u.to_string(), "http://user@h.com:81/a/b?k=v%20w#f");
    URI c = u;  // copies keep the raw query and the parsed view
    EXPECT_EQ(*c.GetQuery("k"), "v w");
    c.SetQuery("k", "z");
    EXPECT_EQ(*u.GetQuery("k"), "v w");
    EXPECT_EQ(c.query(), "k=z");
}

TEST(UriDepth, queries_view_and_valid_characters) {
    URI u;
    ASSERT_EQ(u.SetHttpURL("/p?b=2&a=1&c=%2Fx"), 0);
    const auto m = u.queries();
    ASSERT_EQ(m.size(), 3u);
    EXPECT_EQ(m.at("c"), "/x");
    // every printable, non-space character is allowed in each part
    std::string all;
    for (int c = 0x21; c < 0x7f; ++c) {
        if (c != '#' && c != '?' && c != '&' && c != '=') all.push_back((char)c);
    }
    EXPECT_EQ(u.SetHttpURL("/" + all), 0);
    EXPECT_EQ(u.SetHttpURL("/p?k=" + all), 0);
    EXPECT_EQ(u.SetHttpURL("/p#" + all + "?&="), 0);
}
