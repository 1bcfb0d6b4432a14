#!/usr/bin/env python3
"""SIMT divergence of the step's loops, measured on the host build of the device rule code.

    python3 tools/simt_divergence.py [--boards 32768 --steps 12]

Copies element-crush-gym_amd/csrc/m3_*.hpp into a temp dir, inserts counting
hooks at the loops of apply_action (run starts of the match scan, special
triggers, gravity drop passes, refill draws, spawn groups, cascade iterations),
compiles a small g++ driver and plays seeded random-action episodes (exact
FullMT path). For waves of 64 consecutive boards it reports, per loop, the mean
trips per board and the trips a wave executes (the max over its lanes, per
cascade iteration), i.e. the SIMT efficiency the one-board-per-lane kernels
get; and the effect of bounding k_env_step's cascade (LIM iterations) and its
refill size (HMAX holes). Measurement tool only: never part of the library.
"""
import argparse
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "element-crush-gym_amd", "csrc")

HOOK_H = r'''#pragma once
#include <map>
#include <tuple>
#include <vector>
struct SimLane { int iter = 0; std::vector<int> holes; std::map<std::tuple<int, int>, int> trips; };
extern SimLane* g_sim;
#define SIM_TRIP(id) do { if (g_sim) g_sim->trips[std::make_tuple(g_sim->iter, id)]++; } while (0)
#define SIM_ITER() do { if (g_sim) g_sim->iter++; } while (0)
#define SIM_HOLES(x) do { if (g_sim) g_sim->holes.push_back(x); } while (0)
'''

DRIVER = r'''#include "m3_rules.hpp"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
using namespace m3;
SimLane* g_sim = nullptr;
using CF = Cfg<9, 9, 6>;
using Bd = CF::Bd;
struct Store { static constexpr int CAP = CF::MAXG; Bd h[CF::MAXG], v[CF::MAXG];
  Bd get_h(int g) const { return h[g]; } Bd get_v(int g) const { return v[g]; }
  bool put(int g, const Bd& hh, const Bd& vv) { h[g] = hh; v[g] = vv; return true; } };
int main(int argc, char** argv) {
  const int nb = atoi(argv[1]) / 64 * 64, steps = atoi(argv[2]);
  std::vector<SimLane> lanes(nb);
  std::vector<Bd> boards(nb * CF::NP);
  std::vector<uint32_t> seeds(nb);
  std::vector<int> nact(nb);
  for (int i = 0; i < nb; ++i) {
    seeds[i] = 1000 + i;
    FullMT* fm = new FullMT; fm->init(seeds[i], 0);
    { NoStore ns; init_board<CF>(&boards[i * CF::NP], *fm, ns); } delete fm;
    Bd HL, VL; legal_masks<CF>(&boards[i * CF::NP], special_mask<CF, CF::NP>(&boards[i * CF::NP]), HL, VL);
    uint32_t act[CF::AW]; action_bits<CF>(HL, VL, act);
    ChainMT r; r.init(seeds[i], mt_state397(seeds[i]));
    nact[i] = random_action<CF>(act, r);
  }
  std::map<int, double> lane_trips, wave_trips;
  double lane_iters = 0, wave_iters = 0;
  const int LIMS[2] = {2, 3}, HMAXS[4] = {81, 12, 9, 7};
  double b_wtr[2][4] = {}, b_ltr[2][4] = {}, b_paused[2][4] = {};
  for (int t = 0; t < steps; ++t) {
    for (int i = 0; i < nb; ++i) {
      lanes[i] = SimLane(); g_sim = &lanes[i];
      FullMT* fm = new FullMT; fm->init(seeds[i], 0);
      Store* st = new Store;
      uint32_t f; Bd HL, VL;
      apply_action<CF>(&boards[i * CF::NP], 20 - t, nact[i], *fm, f, HL, VL, *st);
      g_sim = nullptr;
      uint32_t act[CF::AW]; action_bits<CF>(HL, VL, act);
      nact[i] = random_action<CF>(act, *fm);
      delete fm; delete st;
    }
    for (int w = 0; w < nb / 64; ++w) {
      std::map<std::tuple<int, int>, int> mx; int mi = 0;
      for (int l = 0; l < 64; ++l) {
        SimLane& L = lanes[w * 64 + l];
        lane_iters += L.iter; mi = std::max(mi, L.iter);
        for (auto& kv : L.trips) { mx[kv.first] = std::max(mx[kv.first], kv.second); lane_trips[std::get<1>(kv.first)] += kv.second; }
      }
      wave_iters += mi;
      for (auto& kv : mx) wave_trips[std::get<1>(kv.first)] += kv.second;
      for (int li = 0; li < 2; ++li) for (int hi = 0; hi < 4; ++hi) {
        std::map<int, int> m2;
        for (int l = 0; l < 64; ++l) {
          SimLane& L = lanes[w * 64 + l];
          int k = 0;
          while (k < L.iter && k < LIMS[li] && L.holes[k] <= HMAXS[hi]) ++k;
          if (k < L.iter) b_paused[li][hi]++;
          for (int j = 0; j < k; ++j) { int tr = L.trips[std::make_tuple(j + 1, 4)]; m2[j] = std::max(m2[j], tr); b_ltr[li][hi] += tr; }
        }
        for (auto& kv : m2) b_wtr[li][hi] += kv.second;
      }
    }
  }
  const double waves = (double)nb / 64 * steps, lanes_n = (double)nb * steps;
  printf("cascade iterations: per board %.2f, per wave (max over lanes) %.2f\n", lane_iters / lanes_n, wave_iters / waves);
  const char* names[] = {"", "match run starts", "special triggers", "gravity passes/stages", "refill draws", "spawn groups", "group search"};
  for (auto& kv : wave_trips)
    printf("%-17s per board %6.2f  per wave %6.2f  SIMT efficiency %.2f\n", names[kv.first],
           lane_trips[kv.first] / lanes_n, kv.second / waves, lane_trips[kv.first] / (kv.second * 64));
  printf("k_env_step bound (LIM cascade iterations, refills of <= HMAX holes): refill draws per wave / per board, share paused\n");
  for (int li = 0; li < 2; ++li) for (int hi = 0; hi < 4; ++hi)
    printf("  LIM %d HMAX %2d: %6.1f / %5.1f  paused %.3f\n", LIMS[li], HMAXS[hi], b_wtr[li][hi] / waves,
           b_ltr[li][hi] / lanes_n, b_paused[li][hi] / lanes_n);
}
'''

PATCHES = [  # (anchor, text inserted after it)
    ("    while (cand.any()) {                                       // row-major scan over run starts", "\n        SIM_TRIP(1);"),
    ("    while (trig.any()) {\n        const int x = trig.lowest();", "\n        SIM_TRIP(2);"),
    ("    for (;;) {  // drop every tile that has a hole somewhere below it by one row", "\n        SIM_TRIP(3);"),
    # round 5: the decomposed gravity -- a stage counts for a lane that still has holes to close
    ("        constexpr int D = (1 << decltype(S)::value) * C;  // rows moved in this stage, as bits",
     "\n        if (mk.any()) SIM_TRIP(3);"),
    ("        uint32_t v = rng.next32() & tmask;", "\n        SIM_TRIP(4);"),
    ("        for (int gi = 0; gi < ng; ++gi) {                      // get_match_spawn_mask (:159-169)", "\n            SIM_TRIP(5);"),
    ("                    if ((st.get_v(gi) & rh).any()) { g = gi; break; }", "\n                    SIM_TRIP(6);"),
    ("                ++it;\n                const Bd em = gravity<CF>(P, dm);               // :166-173",
     "\n                SIM_ITER();\n                SIM_HOLES(VALID.andnot(tb_nonzero<CF>(P) | special_mask<CF, 6>(P)).popc());"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--boards", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=12)
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="m3simt_")
    try:
        for f in ("m3_rules.hpp", "m3_bitboard.hpp", "m3_rng.hpp"):
            shutil.copy(os.path.join(CSRC, f), d)
        p = os.path.join(d, "m3_rules.hpp")
        s = open(p).read().replace("namespace m3 {", '#include "simhook.h"\nnamespace m3 {', 1)
        for anchor, text in PATCHES:
            assert s.count(anchor) == 1, f"hook anchor not found (m3_rules.hpp changed?): {anchor[:60]!r}"
            s = s.replace(anchor, anchor + text)
        open(p, "w").write(s)
        open(os.path.join(d, "simhook.h"), "w").write(HOOK_H)
        open(os.path.join(d, "sim.cpp"), "w").write(DRIVER)
        subprocess.run(["g++", "-O2", "-std=c++17", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", "-x", "c++",
                        os.path.join(d, "sim.cpp"), "-o", os.path.join(d, "sim")], check=True)
        subprocess.run([os.path.join(d, "sim"), str(a.boards), str(a.steps)], check=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
