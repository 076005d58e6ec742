for rep in 1 2; do for v in g256 g512 g128; do
RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python3 bench.py --feature bias --steps 10 --warmup 2 --profile-only 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(\"$v\", d[\"ms_per_step\"], d[\"kernels_ms\"][\"tail_after_base\"])"
done; done
