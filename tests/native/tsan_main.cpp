// TEST-ONLY race check of the product's host code under ThreadSanitizer
// (tests/test_tsan.py builds this with -fsanitize=thread): the way the job
// engine drives it -- several caller threads planning batches on ONE shared
// WorkPool (engine.hip's dispatcher + staged batches + the prover slots), the
// flat layout / blob write, and the idemix and token-request decoders running
// concurrently.  Every concurrent plan must equal the single-threaded one byte
// for byte.  Input: a file of records [u32 kind][u32 n_in][u32 n_out][u32 len]
// [inputs][outputs][proof] written by the test, and the PP JSON.
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "../../fabric-token-sdk_amd/csrc/host/idemix.h"
#include "../../fabric-token-sdk_amd/csrc/host/planner.h"
#include "../../fabric-token-sdk_amd/csrc/host/request.h"

using namespace ftsh;

static std::vector<uint8_t> slurp(const char* path) {
  std::vector<uint8_t> b;
  FILE* f = fopen(path, "rb");
  if (!f) return b;
  uint8_t buf[65536];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + k);
  fclose(f);
  return b;
}

static std::vector<uint8_t> plan_blob(const PPInfo& pp, const std::vector<PlanItem>& items, WorkPool& pool,
                                      const std::vector<uint8_t>& cbytes) {
  PlanWork w;
  plan_items(pp, items.size(), items.data(), w, pool);
  FlatPlan fp;
  std::string e = flat_layout(w, false, fp);
  if (!e.empty()) return {};
  std::vector<uint8_t> blob(fp.bytes);
  flat_write(w, fp, blob.data(), cbytes.data(), pool);
  return blob;
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  std::vector<uint8_t> ppj = slurp(argv[1]), recs = slurp(argv[2]), owners = slurp(argv[3]);
  PPInfo pp;
  std::string e = parse_pp(ppj.data(), ppj.size(), "zkatdlog", pp);
  if (!e.empty()) {
    fprintf(stderr, "pp: %s\n", e.c_str());
    return 2;
  }
  std::vector<PlanItem> items;
  for (size_t o = 0; o + 16 <= recs.size();) {
    uint32_t h[4];
    memcpy(h, &recs[o], 16);
    o += 16;
    PlanItem it;
    memset(&it, 0, sizeof it);
    it.kind = 0;
    it.t = {&recs[o], h[1], &recs[o + 64 * h[1]], h[2], &recs[o + 64 * (h[1] + h[2])], h[3]};
    o += 64 * (h[1] + h[2]) + h[3];
    items.push_back(it);
  }
  std::vector<uint8_t> cbytes(1 << 16, 0);
  WorkPool pool(4);
  std::vector<uint8_t> want = plan_blob(pp, items, pool, cbytes);
  if (want.empty()) return 3;
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 6; t++)
    th.emplace_back([&, t]() {
      for (int r = 0; r < 3; r++) {
        if (t < 4) {
          if (plan_blob(pp, items, pool, cbytes) != want) bad++;
        } else {
          // owner-signature and request decoding on their own threads (records:
          // [u32 owner_len][u32 sig_len][owner][sig])
          for (size_t o = 0; o + 8 <= owners.size();) {
            uint32_t h[2];
            memcpy(h, &owners[o], 8);
            o += 8;
            NymDecoded d;
            decode_owner_signature(&owners[o], h[0], &owners[o + h[0]], h[1], d);
            o += h[0] + h[1];
          }
          std::vector<Slice> f[4];
          (void)der_token_request(recs.data(), recs.size() < 300 ? recs.size() : 300, f);
        }
      }
    });
  for (auto& x : th) x.join();
  printf("items %zu blob %zu mismatches %d\n", items.size(), want.size(), bad.load());
  return bad.load() ? 1 : 0;
}
