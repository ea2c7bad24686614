"""Generate tests/golden/mt19937_gcc11.json from the REAL libstdc++ of this
container (GCC 11): std::mt19937(seed) raw outputs and
std::uniform_int_distribution<int>(0, INT_MAX) draws — the exact call opengv's
SampleConsensusProblem makes (SURVEY.md §0 finding 5) — and small-range draws
(0, n-1), dpgo_ros's uniform choice of the executing robot. Run: python gen_mt19937_gcc11.py"""
import json, os, subprocess, tempfile
from pathlib import Path

SRC = r'''
#include <climits>
#include <cstdio>
#include <random>
int main() {
  for (unsigned seed : {12345u, 5489u, 1u}) {
    std::mt19937 raw(seed);
    std::printf("raw %u", seed);
    for (int i = 0; i < 2000; ++i) std::printf(" %u", (unsigned)raw());
    std::printf("\n");
    std::mt19937 eng(seed);
    std::uniform_int_distribution<> dist(0, std::numeric_limits<int>::max());
    std::printf("uid %u", seed);
    for (int i = 0; i < 2000; ++i) std::printf(" %d", dist(eng));
    std::printf("\n");
  }
  // small ranges: dpgo_ros's uniform choice of the next executing robot
  for (unsigned seed : {0u, 7u})
    for (int n : {2, 3, 6, 8, 13}) {
      std::mt19937 eng(seed);
      std::printf("small %u:%d", seed, n);
      for (int i = 0; i < 200; ++i) {
        std::uniform_int_distribution<int> pick(0, n - 1);
        std::printf(" %d", pick(eng));
      }
      std::printf("\n");
    }
  std::mt19937 kat;  // default seed 5489: the standard's 10000th-output check
  unsigned v = 0;
  for (int i = 0; i < 10000; ++i) v = (unsigned)kat();
  std::printf("kat %u\n", v);
  std::printf("gcc %d\n", __GNUC__);
}
'''

def main():
    here = Path(__file__).resolve().parent
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "g.cpp"), os.path.join(d, "g")
        open(src, "w").write(SRC)
        subprocess.run(["g++", "-O2", "-std=c++17", src, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split("\n")
    res = {"raw": {}, "uid": {}, "small": {}}
    for line in out:
        if not line:
            continue
        tok = line.split()
        if tok[0] in ("raw", "uid", "small"):
            res[tok[0]][tok[1]] = [int(x) for x in tok[2:]]
        elif tok[0] == "kat":
            res["kat_10000"] = int(tok[1])
        elif tok[0] == "gcc":
            res["gcc_major"] = int(tok[1])
    (here / "mt19937_gcc11.json").write_text(json.dumps(res))

if __name__ == "__main__":
    main()
