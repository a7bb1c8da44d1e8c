// Diagnostic (not product, not a test): how many PARITY E-step records can
// never change their float accumulator?  Reuses the CPU oracle's lattice.
//
// A record c >= 0 added to a float e >= e_lb > 0 as e = (float)((double)e + c)
// leaves e unchanged when c < ulp(e_lb) / 4 (the double sum is within
// ulp/4 + 2^-52 ulp of e, so the float rounding returns e).  e only grows, so
// the accumulator's value at any earlier time is such a lower bound.  This
// tool runs the RunEStep bucket emulation (T buckets, chunks of C sentences,
// the lower bound = each key's value at its chunk's start) and counts records
// below the bound: (a) per (bucket, id) key, (b) per id with the bound = the
// minimum over buckets, only for the H highest-score ids (an LDS table).
// It also re-runs the accumulation with the dropped records skipped and checks
// the result is bit-identical.
//
// Build: g++ -O2 -std=c++17 -ffp-contract=off -pthread tools/estep_drop_census.cc -o /tmp/census
// Input files (tools/estep_drop_census.py writes them): sent.bin sent_off.bin
// pieces.bin piece_off.bin scores.bin in DIR.
#include "../oracle/spm_oracle.cc"

#include <cstdio>
#include <fstream>
#include <iterator>

using namespace oracle;

static std::vector<char> ReadAll(const std::string &p) {
  std::ifstream f(p, std::ios::binary);
  return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static double Thr(float e) {  // ulp(e)/4 for a positive normal float, else 0
  uint32_t b;
  std::memcpy(&b, &e, 4);
  const int ex = (b >> 23) & 0xFF;
  if (ex == 0 || ex == 0xFF || (b >> 31)) return 0.0;
  return std::ldexp(1.0, ex - 127 - 25);
}

int main(int argc, char **argv) {
  const std::string dir = argv[1];
  const int T = argc > 2 ? atoi(argv[2]) : 16;
  const uint64_t C = argc > 3 ? strtoull(argv[3], nullptr, 10) : 3125000;
  const int H = argc > 4 ? atoi(argv[4]) : 4096;
  const int reps = argc > 5 ? atoi(argv[5]) : 1;
  auto sb = ReadAll(dir + "/sent.bin");
  auto so = ReadAll(dir + "/sent_off.bin");
  auto pb = ReadAll(dir + "/pieces.bin");
  auto po = ReadAll(dir + "/piece_off.bin");
  auto sc = ReadAll(dir + "/scores.bin");
  const uint64_t *off = reinterpret_cast<const uint64_t *>(so.data());
  const uint64_t n0 = so.size() / 8 - 1;
  const uint64_t *poff = reinterpret_cast<const uint64_t *>(po.data());
  const uint64_t V = po.size() / 8 - 1;
  const float *scores = reinterpret_cast<const float *>(sc.data());
  ByteTrie trie;
  std::vector<float> scv(scores, scores + V);
  float min_score = FLT_MAX;
  for (uint64_t i = 0; i < V; ++i) {
    trie.Insert(std::string(pb.data() + poff[i], poff[i + 1] - poff[i]), int(i));
    min_score = std::min(min_score, scores[i]);
  }
  UnigramScoring m{&trie, &scv, nullptr, min_score, 0.0f, 0};
  // Hot ids: the H highest scores (FAST mode's LDS table rule).
  std::vector<int> order(V);
  for (uint64_t i = 0; i < V; ++i) order[i] = int(i);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return scores[a] > scores[b]; });
  std::vector<char> hot(V, 0);
  for (int k = 0; k < H && k < int(V); ++k) hot[order[k]] = 1;
  const uint64_t n = n0 * reps;  // sentence g = buffer g % n0 (the bench's re-used buffer)
  std::vector<std::vector<float>> e(T, std::vector<float>(V, 0.f)), e2(T, std::vector<float>(V, 0.f));
  std::vector<uint64_t> rec(T, 0), drop_key(T, 0), drop_id(T, 0);
  std::vector<double> id_thr(V, 0.0);
  for (uint64_t c0 = 0; c0 < n; c0 += C) {
    const uint64_t c1 = std::min(n, c0 + C);
    // Chunk-start lower bounds.
    std::vector<std::vector<double>> kthr(T, std::vector<double>(V));
    for (int t = 0; t < T; ++t)
      for (uint64_t v = 0; v < V; ++v) kthr[t][v] = Thr(e[t][v]);
    for (uint64_t v = 0; v < V; ++v) {
      double mn = 1e300;
      for (int t = 0; t < T; ++t) mn = std::min(mn, kthr[t][v]);
      id_thr[v] = hot[v] ? mn : 0.0;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        Lattice L;
        uint64_t first = c0 + ((t - c0 % T) % T + T) % T;
        for (uint64_t g = first; g < c1; g += T) {
          const uint64_t i = g % n0;
          const char *s = sb.data() + off[i];
          const size_t len = off[i + 1] - off[i];
          L.SetSentence(s, len);
          PopulateNodes(m, s, &L);
          const float f = 1.0f;
          // PopulateMarginal with the per-record census.
          const int lenc = L.size();
          std::vector<float> alpha(L.nodes.size(), 0.0f), beta(L.nodes.size(), 0.0f);
          for (int pos = 0; pos <= lenc; ++pos)
            for (int r : L.begin_nodes[pos])
              for (int l : L.end_nodes[pos])
                alpha[r] = LogSumExp(alpha[r], L.nodes[l].score + alpha[l], l == L.end_nodes[pos][0]);
          for (int pos = lenc; pos >= 0; --pos)
            for (int l : L.end_nodes[pos])
              for (int r : L.begin_nodes[pos])
                beta[l] = LogSumExp(beta[l], L.nodes[r].score + beta[r], r == L.begin_nodes[pos][0]);
          const float Z = alpha[L.begin_nodes[lenc][0]];
          for (int pos = 0; pos < lenc; ++pos)
            for (int nd : L.begin_nodes[pos]) {
              const auto &nn = L.nodes[nd];
              const float a = alpha[nd] + nn.score + beta[nd] - Z;
              const double c = f * exp(double(a));
              e[t][nn.id] = static_cast<float>(static_cast<double>(e[t][nn.id]) + c);
              ++rec[t];
              const bool dk = c < kthr[t][nn.id];
              if (dk) ++drop_key[t];
              if (c < id_thr[nn.id]) ++drop_id[t];
              if (!dk) e2[t][nn.id] = static_cast<float>(static_cast<double>(e2[t][nn.id]) + c);
            }
        }
      });
    for (auto &x : th) x.join();
    uint64_t R = 0, DK = 0, DI = 0;
    for (int t = 0; t < T; ++t) R += rec[t], DK += drop_key[t], DI += drop_id[t];
    fprintf(stderr, "chunk @%llu: records %llu, droppable per key %.3f, per hot id %.3f\n",
            (unsigned long long)c0, (unsigned long long)R, double(DK) / R, double(DI) / R);
  }
  uint64_t bad = 0;
  for (int t = 0; t < T; ++t)
    for (uint64_t v = 0; v < V; ++v) bad += std::memcmp(&e[t][v], &e2[t][v], 4) != 0;
  uint64_t R = 0, DK = 0, DI = 0;
  for (int t = 0; t < T; ++t) R += rec[t], DK += drop_key[t], DI += drop_id[t];
  printf("{\"sentences\": %llu, \"T\": %d, \"chunk\": %llu, \"records\": %llu, \"records_per_sentence\": %.2f, "
         "\"drop_key_frac\": %.4f, \"drop_hot_id_frac\": %.4f, \"hot\": %d, \"mismatch_after_drop\": %llu}\n",
         (unsigned long long)n, T, (unsigned long long)C, (unsigned long long)R, double(R) / n, double(DK) / R,
         double(DI) / R, H, (unsigned long long)bad);
  return 0;
}
