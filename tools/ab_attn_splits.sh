# A/B of the attention split count (GRL_ATTN_SPLITS=S forces S; "auto" = the
# library's rule, attn_splits in attention.hip).
# Usage: bash tools/ab_attn_splits.sh "auto 1 3 7" N...
vals=${1:-"auto 1 3 5 7"}; shift
for r in 1 2; do
  for s in $vals; do
    if [ "$s" = auto ]; then
      echo "splits $s: $(timeout -k 10 200 python tools/probe_attn.py "$@" 2>/dev/null | tr '\n' ' ')"
    else
      echo "splits $s: $(GRL_ATTN_SPLITS=$s timeout -k 10 200 python tools/probe_attn.py "$@" 2>/dev/null | tr '\n' ' ')"
    fi
  done
done
