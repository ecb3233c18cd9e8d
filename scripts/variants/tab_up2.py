# A/B: 2 gathers in flight a lane in the tab kernels' layer 2 (kTabUP) instead of 4.
EDITS = [("segspmm.hip", "constexpr int kTabUP = 4;", "constexpr int kTabUP = 2;")]
