# epilogue_row with 4 partial loads in flight a lane (default 8)
EDITS = [("spmm.hip", "constexpr int kEpiBatch = 8;", "constexpr int kEpiBatch = 4;")]
