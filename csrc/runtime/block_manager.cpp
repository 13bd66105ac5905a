// Paged KV-cache block allocator + per-step metadata builders (host C++).
//
// Replaces HF's per-request `past_key_values` tensors (grown by torch.cat every step,
// SURVEY.md §2.4 K6) with a fixed pool of `num_blocks` blocks of `block_size` tokens per
// layer, sized from HBM at engine start (288 GB per MI355X => millions of tokens). The
// scheduler (Python) asks this allocator for blocks; the batch builders below emit the
// int32 block tables and slot mappings the HIP kernels consume, so per-step metadata for a
// 256-sequence batch is built without a Python loop over tokens.
//
// C ABI (ctypes): every function returns >= 0 on success, negative on failure.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

struct BlockManager {
  int num_blocks;
  int block_size;
  std::vector<int> free_list;                              // stack of free block ids
  std::unordered_map<long long, std::vector<int>> tables;  // seq id -> blocks
  // automatic prefix caching: a FULL block whose tokens (and all tokens before them) are
  // known carries a chain hash; a later sequence with the same prefix maps the same block
  // (refcount) instead of recomputing its KV. A block released by its last user keeps its
  // hash and content and waits in `evictable` (oldest first) until the pool runs dry.
  std::vector<int> refcnt;
  std::vector<unsigned long long> hash_of;                 // 0 = no hash
  std::unordered_map<unsigned long long, int> cached;      // hash -> block
  std::deque<int> evictable;                               // lazily pruned (refcnt > 0)
  int n_evictable = 0;
  long long hits = 0;                                      // blocks served from the cache
  std::mutex mu;

  BlockManager(int nb, int bs)
      : num_blocks(nb), block_size(bs), refcnt(nb, 0), hash_of(nb, 0ull) {
    free_list.reserve(nb);
    // hand out low block ids first (LIFO stack, reversed fill)
    for (int b = nb - 1; b >= 0; --b) free_list.push_back(b);
  }
  int blocks_for(long long tokens) const {
    return (int)((tokens + block_size - 1) / block_size);
  }
  int available() const { return (int)free_list.size() + n_evictable; }
  // a block for exclusive use: a never-hashed free one first, else evict the oldest cached
  int alloc() {
    if (!free_list.empty()) {
      const int b = free_list.back();
      free_list.pop_back();
      refcnt[b] = 1;
      return b;
    }
    while (!evictable.empty()) {
      const int b = evictable.front();
      evictable.pop_front();
      if (refcnt[b] != 0 || hash_of[b] == 0) continue;       // revived / stale entry
      cached.erase(hash_of[b]);
      hash_of[b] = 0;
      --n_evictable;
      refcnt[b] = 1;
      return b;
    }
    return -1;
  }
  void release(int b) {
    if (--refcnt[b] > 0) return;
    if (hash_of[b] != 0) {
      evictable.push_back(b);
      ++n_evictable;
    } else {
      free_list.push_back(b);
    }
  }
  bool grow(std::vector<int>& tab, int need) {               // all-or-nothing
    if (available() < need) return false;
    for (int i = 0; i < need; ++i) tab.push_back(alloc());
    return true;
  }
};

inline BlockManager* H(void* h) { return reinterpret_cast<BlockManager*>(h); }

}  // namespace

extern "C" {

void* dli_bm_create(int num_blocks, int block_size) {
  if (num_blocks <= 0 || block_size <= 0) return nullptr;
  return new BlockManager(num_blocks, block_size);
}

void dli_bm_destroy(void* h) { delete H(h); }

int dli_bm_num_free(void* h) {
  std::lock_guard<std::mutex> g(H(h)->mu);
  return H(h)->available();
}

int dli_bm_num_blocks(void* h) { return H(h)->num_blocks; }
int dli_bm_block_size(void* h) { return H(h)->block_size; }

// Blocks still needed so that `seq` covers `total_tokens` tokens.
int dli_bm_blocks_needed(void* h, long long seq, long long total_tokens) {
  auto* m = H(h);
  std::lock_guard<std::mutex> g(m->mu);
  auto it = m->tables.find(seq);
  const int have = it == m->tables.end() ? 0 : (int)it->second.size();
  return std::max(0, m->blocks_for(total_tokens) - have);
}

// Grow `seq`'s table to cover `total_tokens`; all-or-nothing. Returns blocks added or -1.
int dli_bm_ensure(void* h, long long seq, long long total_tokens) {
  auto* m = H(h);
  std::lock_guard<std::mutex> g(m->mu);
  auto& tab = m->tables[seq];
  const int need = m->blocks_for(total_tokens) - (int)tab.size();
  if (need <= 0) return 0;
  if (!m->grow(tab, need)) {
    if (tab.empty()) m->tables.erase(seq);
    return -1;
  }
  return need;
}

// ensure() for (seqs[i], totals[i]) in order; stops at the first sequence that does not
// fit. Returns how many succeeded.
int dli_bm_ensure_batch(void* h, const long long* seqs, const int* totals, int n) {
  auto* m = H(h);
  std::lock_guard<std::mutex> g(m->mu);
  for (int i = 0; i < n; ++i) {
    auto& tab = m->tables[seqs[i]];
    const int need = m->blocks_for(totals[i]) - (int)tab.size();
    if (need <= 0) continue;
    if (!m->grow(tab, need)) {
      if (tab.empty()) m->tables.erase(seqs[i]);
      return i;
    }
  }
  return n;
}

// Release every block of `seq`. Returns the number released.
int dli_bm_free(void* h, long long seq) {
  auto* m = H(h);
  std::lock_guard<std::mutex> g(m->mu);
  auto it = m->tables.find(seq);
  if (it == m->tables.end()) return 0;
  const int n = (int)it->second.size();
  for (auto it2 = it->second.rbegin(); it2 != it->second.rend(); ++it2) m->release(*it2);
  m->tables.erase(it);
  return n;
}

// dli_bm_free for seqs[0..n); returns the blocks released.
int dli_bm_free_batch(void* h, const long long* seqs, int n) {
  auto* m = H(h);
  std::lock_guard<std::mutex> g(m->mu);
  int total = 0;
  for (int i = 0; i < n; ++i) {
    auto it = m->tables.find(seqs[i]);
    if (it == m->tables.end()) continue;
    total += (int)it->second.size();
    for (auto it2 = it->second.rbegin(); it2 != it->second.rend(); ++it2) m->release(*it2);
    m->tables.erase(it);
  }
  return total;
}

int dli_bm_table(void* h, long long seq, int* out, int max_blocks) {
  auto* m = H(h);
  std::lock_guard<std::mutex> g(m->mu);
  auto it = m->tables.find(seq);
  if (it == m->tables.end()) return 0;
  const int n = std::min((int)it->second.size(), max_blocks);
  std::memcpy(out, it->second.data(), sizeof(int) * n);
  return n;
}

// Padded [n, max_blocks] block tables (pad = 0: a valid block id that kernels never read
// past context_lens). Returns the widest table or -1 if a table exceeds max_blocks.
int dli_bm_fill_tables(void* h, const long long* seqs, int n, int* out, int max_blocks) {
  auto* m = H(h);
  std::lock_guard<std::mutex> g(m->mu);
  int widest = 0;
  for (int i = 0; i < n; ++i) {
    int* row = out + (long)i * max_blocks;
    auto it = m->tables.find(seqs[i]);
    int cnt = 0;
    if (it != m->tables.end()) {
      cnt = (int)it->second.size();
      if (cnt > max_blocks) return -1;
      std::memcpy(row, it->second.data(), sizeof(int) * cnt);
    }
    std::fill(row + cnt, row + max_blocks, 0);
    widest = std::max(widest, cnt);
  }
  return widest;
}

// One decode step's KV metadata in a single call (the per-tick hot path of the scheduler):
// for each sequence i, grow its table to cover ctx[i] tokens (the new token is at position
// ctx[i] - 1), write that token's slot to slots[i] and the padded table row to
// tables[i * max_blocks ...]. Returns the widest table, or -(i + 1) if sequence i could not
// get a block (earlier sequences keep theirs: they need them anyway), or -(n + 1) if a
// table exceeds max_blocks.
int dli_bm_decode_prepare(void* h, const long long* seqs, const int* ctx, int n, int* slots,
                          int* tables, int max_blocks) {
  auto* m = H(h);
  std::lock_guard<std::mutex> g(m->mu);
  const int bs = m->block_size;
  int widest = 0;
  for (int i = 0; i < n; ++i) {
    auto& tab = m->tables[seqs[i]];
    const int need = m->blocks_for(ctx[i]) - (int)tab.size();
    if (need > 0 && !m->grow(tab, need)) {
      if (tab.empty()) m->tables.erase(seqs[i]);
      return -(i + 1);
    }
    const int cnt = (int)tab.size();
    if (cnt > max_blocks) return -(n + 1);
    const int t = ctx[i] - 1;
    slots[i] = tab[t / bs] * bs + (t % bs);
    int* row = tables + (long)i * max_blocks;
    std::memcpy(row, tab.data(), sizeof(int) * cnt);
    std::fill(row + cnt, row + max_blocks, 0);
    widest = std::max(widest, cnt);
  }
  return widest;
}

// slot ids for tokens [start_i, start_i + count_i) of each sequence, concatenated.
int dli_bm_slot_mapping(void* h, const long long* seqs, const int* starts, const int* counts,
                        int n, int* out) {
  auto* m = H(h);
  std::lock_guard<std::mutex> g(m->mu);
  long o = 0;
  const int bs = m->block_size;
  for (int i = 0; i < n; ++i) {
    auto it = m->tables.find(seqs[i]);
    if (it == m->tables.end()) return -1;
    const auto& tab = it->second;
    for (int t = starts[i]; t < starts[i] + counts[i]; ++t) {
      const int b = t / bs;
      if (b >= (int)tab.size()) return -1;
      out[o++] = tab[b] * bs + (t % bs);
    }
  }
  return (int)o;
}

// Prefix caching. A new sequence `seq` (no blocks yet) maps the longest run of cached blocks
// whose chain hashes are hashes[0..n): returns the number of blocks mapped (their tokens need
// no prefill). Each mapped block gains a reference.
int dli_bm_match_prefix(void* h, long long seq, const unsigned long long* hashes, int n) {
  auto* m = H(h);
  std::lock_guard<std::mutex> g(m->mu);
  auto& tab = m->tables[seq];
  if (!tab.empty()) return 0;
  int k = 0;
  for (; k < n; ++k) {
    auto it = m->cached.find(hashes[k]);
    if (it == m->cached.end()) break;
    const int b = it->second;
    if (m->refcnt[b] == 0) --m->n_evictable;                // revived (queue entry goes stale)
    ++m->refcnt[b];
    tab.push_back(b);
  }
  if (tab.empty()) m->tables.erase(seq);
  m->hits += k;
  return k;
}

// Publish blocks [first, first + n) of `seq` (their KV is written by a step already queued
// on the device) under hashes[0..n) so later sequences can map them. A hash that is already
// cached (another sequence computed the same prefix) is left alone. Returns blocks added.
int dli_bm_register_prefix(void* h, long long seq, const unsigned long long* hashes,
                           int first, int n) {
  auto* m = H(h);
  std::lock_guard<std::mutex> g(m->mu);
  auto it = m->tables.find(seq);
  if (it == m->tables.end()) return 0;
  const auto& tab = it->second;
  int added = 0;
  for (int k = 0; k < n && first + k < (int)tab.size(); ++k) {
    const int b = tab[first + k];
    const unsigned long long hv = hashes[k];
    if (hv == 0 || m->hash_of[b] != 0 || m->cached.count(hv)) continue;
    m->hash_of[b] = hv;
    m->cached[hv] = b;
    ++added;
  }
  return added;
}

long long dli_bm_prefix_hits(void* h) {
  std::lock_guard<std::mutex> g(H(h)->mu);
  return H(h)->hits;
}

int dli_bm_num_cached(void* h) {
  std::lock_guard<std::mutex> g(H(h)->mu);
  return (int)H(h)->cached.size();
}

}  // extern "C"
