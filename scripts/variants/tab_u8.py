# A/B: 8 gathers in flight a lane in the tab kernels' layer 1 (kTabU) instead of 4.
EDITS = [("segspmm.hip", "constexpr int kTabU = 4;", "constexpr int kTabU = 8;")]
