for rep in 1 2; do for v in t16 t24 t32; do
RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python3 bench.py --feature bias --steps 10 --warmup 2 --profile-only 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(\"$v bias\", d[\"ms_per_step\"], d[\"kernels_ms\"][\"tail_after_base\"])"
RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --profile-only 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(\"$v rotate\", d[\"ms_per_step\"], d[\"roofline\"][\"ms\"])"
done; done
