for nb in 1024 768 512; do for mode in static dynamic; do
  MULTIGRAD_FWD_MAX_BLOCKS=$nb MULTIGRAD_LPT=$mode timeout -k 10 300 python tools/kernel_bench.py --tag ${mode}_$nb --params 1250000 --halos 16777216 --iters 50 2>/dev/null | grep tag | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tag'], 'fwd_int', d['fwd_internal_us'], 'blocks', d['fwd_blocks'])"
done; done
