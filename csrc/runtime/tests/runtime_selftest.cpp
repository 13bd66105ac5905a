// Host-side self-test of the C++ runtime (block allocator + safetensors parser), built with
// AddressSanitizer on the host (sanitizers for the C++ layer; GPU ASan is
// not available on this pool). Randomised allocator stress with invariant checks, and a
// parser fuzz: every truncation of a valid header, corrupted length fields and
// out-of-range data offsets must be rejected without any out-of-bounds access.
//
//   build: python -m distributed_llm_inferencing_amd.build --asan-selftest
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <string>
#include <vector>
#include <unistd.h>

extern "C" {
void* dli_bm_create(int, int);
void dli_bm_destroy(void*);
int dli_bm_num_free(void*);
int dli_bm_ensure(void*, long long, long long);
int dli_bm_free(void*, long long);
int dli_bm_table(void*, long long, int*, int);
int dli_bm_fill_tables(void*, const long long*, int, int*, int);
int dli_bm_slot_mapping(void*, const long long*, const int*, const int*, int, int*);
void* dli_st_open(const char*);
void dli_st_close(void*);
int dli_st_count(void*);
int dli_st_info(void*, int, char*, int, char*, int, long long*, int*, long long*);
int dli_st_find(void*, const char*);
int dli_st_copy_to_host(void*, int, void*);
}

static int failures = 0;
#define CHECK(c)                                                             \
  do {                                                                       \
    if (!(c)) { std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++failures; } \
  } while (0)

static void test_block_manager() {
  const int NB = 64, BS = 16, SEQS = 24, W = 16;
  void* bm = dli_bm_create(NB, BS);
  CHECK(bm != nullptr);
  CHECK(dli_bm_create(0, 16) == nullptr);
  std::mt19937 rng(7);
  std::vector<long long> len(SEQS, 0);
  for (int it = 0; it < 20000; ++it) {
    const long long s = rng() % SEQS;
    if (rng() % 3 == 0) {
      dli_bm_free(bm, s);
      len[s] = 0;
    } else {
      const long long want = std::min<long long>(len[s] + 1 + rng() % 40, (long long)W * BS);
      if (dli_bm_ensure(bm, s, want) >= 0) len[s] = want;
    }
    if (it % 97 == 0) {              // invariants: blocks unique, counts add up
      std::set<int> seen;
      int held = 0;
      std::vector<int> tab(W);
      for (int q = 0; q < SEQS; ++q) {
        const int n = dli_bm_table(bm, q, tab.data(), W);
        CHECK(n == (int)((len[q] + BS - 1) / BS) || (len[q] == 0 && n == 0));
        for (int i = 0; i < n; ++i) {
          CHECK(tab[i] >= 0 && tab[i] < NB);
          CHECK(seen.insert(tab[i]).second);
        }
        held += n;
      }
      CHECK(held + dli_bm_num_free(bm) == NB);
      std::vector<long long> seqs(SEQS);
      for (int q = 0; q < SEQS; ++q) seqs[q] = q;
      std::vector<int> tabs(SEQS * W, -1);
      CHECK(dli_bm_fill_tables(bm, seqs.data(), SEQS, tabs.data(), W) >= 0);
      std::vector<int> starts(SEQS, 0), counts(SEQS);
      long long total = 0;
      for (int q = 0; q < SEQS; ++q) { counts[q] = (int)len[q]; total += len[q]; }
      std::vector<int> slots(total + 1);
      std::vector<long long> live;
      std::vector<int> ls, lc;
      for (int q = 0; q < SEQS; ++q)
        if (len[q]) { live.push_back(q); ls.push_back(0); lc.push_back((int)len[q]); }
      const int got = dli_bm_slot_mapping(bm, live.data(), ls.data(), lc.data(),
                                          (int)live.size(), slots.data());
      CHECK(got == (int)total);
      const int one = 1, over = (int)len[live.empty() ? 0 : live[0]] + BS;
      if (!live.empty())             // a token past the table must be rejected
        CHECK(dli_bm_slot_mapping(bm, live.data(), &over, &one, 1, slots.data()) == -1);
    }
  }
  for (int q = 0; q < SEQS; ++q) dli_bm_free(bm, q);
  CHECK(dli_bm_num_free(bm) == NB);
  dli_bm_destroy(bm);
}

static std::string tmpfile_path() {
  char buf[] = "/tmp/dli_st_XXXXXX";
  const int fd = mkstemp(buf);
  if (fd >= 0) close(fd);
  return buf;
}

static void write_file(const std::string& path, uint64_t hlen, const std::string& header,
                       const std::vector<uint8_t>& data) {
  FILE* f = std::fopen(path.c_str(), "wb");
  std::fwrite(&hlen, 8, 1, f);
  std::fwrite(header.data(), 1, header.size(), f);
  if (!data.empty()) std::fwrite(data.data(), 1, data.size(), f);
  std::fclose(f);
}

static void test_safetensors() {
  const std::string hdr =
      "{\"__metadata__\":{\"format\":\"pt\",\"note\":\"a,b}\"},"
      "\"w.a\":{\"dtype\":\"BF16\",\"shape\":[2,3],\"data_offsets\":[0,12]},"
      "\"b\":{\"dtype\":\"I32\",\"shape\":[4],\"data_offsets\":[12,28]},"
      "\"s\":{\"dtype\":\"F32\",\"shape\":[],\"data_offsets\":[28,32]}}";
  std::vector<uint8_t> data(32);
  for (int i = 0; i < 32; ++i) data[i] = (uint8_t)(i * 7 + 1);
  const std::string path = tmpfile_path();
  write_file(path, hdr.size(), hdr, data);
  void* h = dli_st_open(path.c_str());
  CHECK(h != nullptr);
  if (h) {
    CHECK(dli_st_count(h) == 3);
    const int i = dli_st_find(h, "b");
    CHECK(i == 1 && dli_st_find(h, "nope") == -1);
    char name[64], dt[16];
    long long shape[8], nbytes = 0;
    int nd = 0;
    CHECK(dli_st_info(h, i, name, 64, dt, 16, shape, &nd, &nbytes) == 0);
    CHECK(std::string(name) == "b" && std::string(dt) == "I32" && nd == 1 && shape[0] == 4 &&
          nbytes == 16);
    CHECK(dli_st_info(h, 3, name, 64, dt, 16, shape, &nd, &nbytes) == -1);
    uint8_t out[16];
    CHECK(dli_st_copy_to_host(h, i, out) == 0 && std::memcmp(out, data.data() + 12, 16) == 0);
    CHECK(dli_st_copy_to_host(h, -1, out) == -1);
    dli_st_close(h);
  }
  // fuzz: every truncated header (length field = truncated size) must fail cleanly
  int accepted = 0;
  for (size_t cut = 0; cut < hdr.size(); ++cut) {
    write_file(path, cut, hdr.substr(0, cut), {});
    void* g = dli_st_open(path.c_str());
    if (g) { ++accepted; dli_st_close(g); }
  }
  CHECK(accepted == 0);
  // length field past the end of the file, and absurd lengths (overflow attempts)
  for (uint64_t hl : {(uint64_t)hdr.size() + 1, (uint64_t)-1, (uint64_t)-8, (uint64_t)1 << 62}) {
    write_file(path, hl, hdr, {});
    void* g = dli_st_open(path.c_str());
    CHECK(g == nullptr);
    if (g) dli_st_close(g);
  }
  // data offsets outside the data section / inverted
  for (const char* bad : {"[0,33]", "[20,12]", "[-4,4]", "[0,99999999999999999999]"}) {
    std::string hb = "{\"x\":{\"dtype\":\"U8\",\"shape\":[4],\"data_offsets\":";
    hb += bad;
    hb += "}}";
    write_file(path, hb.size(), hb, data);
    void* g = dli_st_open(path.c_str());
    CHECK(g == nullptr);
    if (g) dli_st_close(g);
  }
  CHECK(dli_st_open("/nonexistent/x.safetensors") == nullptr);
  unlink(path.c_str());
}

int main() {
  test_block_manager();
  test_safetensors();
  if (failures) {
    std::fprintf(stderr, "runtime_selftest: %d failure(s)\n", failures);
    return 1;
  }
  std::printf("runtime_selftest: OK\n");
  return 0;
}
