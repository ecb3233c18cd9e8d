# (Adopted in round 6: the tab kernels' lds_ordered_sum is this serial loop; the batched form it
# replaced measured slower — DESIGN §5.)
EDITS = []
