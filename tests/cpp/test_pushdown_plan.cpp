// test_pushdown_plan.cpp — prints rpt::PlanPushdown (include/rpt_host.hpp) for every combination of its inputs, one
// CSV line each; tests/test_pushdown_plan.py checks them against the reference's PushDynamicFilters /
// SetupDynamicFilterPushdown logic restated in Python. Host-only: no device call.
#include <cstdio>

#include "rpt_host.hpp"

int main() {
  for (int dev = 0; dev < 2; dev++)
    for (int ft = 0; ft < 3; ft++)
      for (int fwd = 0; fwd < 2; fwd++)
        for (int tgt = 0; tgt < 2; tgt++)
          for (int rows = 0; rows < 2; rows++)
            for (int bfe = 0; bfe < 2; bfe++)
              for (int mm = 0; mm < 2; mm++) {
                const rpt::PushdownPlan p =
                    rpt::PlanPushdown(dev ? rpt::Device::kGpu : rpt::Device::kCpu, static_cast<rpt::FilterType>(ft),
                                      fwd != 0, tgt != 0, rows ? 1000 : 0, bfe != 0, mm != 0);
                printf("%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d\n", dev, ft, fwd, tgt, rows, bfe, mm, p.use_bf_passthrough,
                       p.push_always_false, p.push_bf, p.push_minmax, p.bf_probed_in_use_bf);
              }
  return 0;
}
