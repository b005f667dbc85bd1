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

// the pipelined token-request path (request.cpp verify_token_requests): chunks
// decoded on `dec` while earlier chunks are "verified" on helper threads that
// plan their transfers on `plan` (as the engine does); the verdicts of a
// pipelined run must equal those of one serial chunk.  Records of argv[4]:
// [u32 kind 0 = request / 1 = ledger entry][u32 key_len][u32 val_len][key][val].
static int request_pipeline(const PPInfo& pp, const std::vector<uint8_t>& recs, WorkPool& plan) {
  std::vector<ftz_bytes> reqs;
  std::vector<std::pair<std::string, std::vector<uint8_t>>> ledger;
  for (size_t o = 0; o + 12 <= recs.size();) {
    uint32_t h[3];
    memcpy(h, &recs[o], 12);
    o += 12;
    if (h[0] == 0) {
      reqs.push_back(ftz_bytes{&recs[o + h[1]], h[2]});
    } else {
      ledger.push_back({std::string((const char*)&recs[o], h[1]), std::vector<uint8_t>(&recs[o + h[1]], &recs[o + h[1] + h[2]])});
    }
    o += h[1] + h[2];
  }
  struct Led {
    const std::vector<std::pair<std::string, std::vector<uint8_t>>>* kv;
  } led{&ledger};
  ftz_get_states_fn gs = [](void* u, size_t n, const ftz_bytes* keys, ftz_bytes* vals) -> int {
    const Led* l = (const Led*)u;
    for (size_t i = 0; i < n; i++) {
      vals[i] = ftz_bytes{nullptr, 0};
      std::string k((const char*)keys[i].p, keys[i].len);
      for (auto& e : *l->kv)
        if (e.first == k) vals[i] = ftz_bytes{e.second.data(), e.second.size()};
    }
    return 0;
  };
  auto run = [&](size_t chunk, size_t inflight, WorkPool* dec, std::vector<int32_t>& codes) {
    RequestHooks h;
    h.check = [](size_t m, const uint8_t*, uint8_t* ok) {
      memset(ok, 1, m);
      return 0;
    };
    // "verification": plan the transfers on the shared planning pool, code = the
    // number of planned pieces mod 7 (deterministic, exercises the planner)
    h.verify_transfers = [&](size_t m, const ftz_transfer* tx, int32_t* c) {
      std::vector<PlanItem> it(m);
      for (size_t i = 0; i < m; i++) {
        memset(&it[i], 0, sizeof it[i]);
        it[i].t = {tx[i].inputs, tx[i].n_in, tx[i].outputs, tx[i].n_out, tx[i].proof, tx[i].proof_len};
      }
      PlanWork w;
      plan_items(pp, m, it.data(), w, plan);
      for (size_t i = 0; i < m; i++) c[i] = (int32_t)((tx[i].proof_len + w.used) % 7);
      return 0;
    };
    h.verify_issues = [](size_t m, const ftz_issue*, int32_t* c) {
      for (size_t i = 0; i < m; i++) c[i] = 0;
      return 0;
    };
    h.get_states = gs;
    h.user = &led;
    h.chunk = chunk;
    h.inflight = inflight;
    if (dec) h.par = [dec](size_t k, const std::function<void(size_t)>& f) { dec->run(k, f); };
    codes.assign(reqs.size(), -1);
    std::vector<int32_t> failed(reqs.size());
    std::string err;
    return verify_token_requests(reqs.size(), reqs.data(), h, codes.data(), failed.data(), err);
  };
  std::vector<int32_t> want, got;
  if (run(1u << 20, 1, nullptr, want) != 0) return -1;
  WorkPool dec(4);
  int bad = 0;
  for (size_t chunk : {1, 3, 7}) {
    if (run(chunk, 4, &dec, got) != 0 || got != want) bad++;
  }
  return bad;
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
  if (argc > 4) {
    int rb = request_pipeline(pp, slurp(argv[4]), pool);
    if (rb < 0) return 4;
    bad += rb;
  }
  printf("items %zu blob %zu mismatches %d\n", items.size(), want.size(), bad.load());
  return bad.load() ? 1 : 0;
}
