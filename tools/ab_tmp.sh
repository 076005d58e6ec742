RNNL_LIB=rnnlogic_amd/_build/variants/new.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "pna or wn or PNA or edge or ranges" > gpurun_out/ab_pytest.log 2>&1; tail -3 gpurun_out/ab_pytest.log
for rep in 1 2; do for v in old old3 new; do
RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python3 tools/wn_profile.py 2>/dev/null | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip().splitlines()[-1]); print(\"$v\", d['ms_per_step'], d['kernels_ms'])"
done; done
for v in old old3 new; do RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 300 python3 tools/interference.py wn 2>/dev/null | grep -E "^\+score |both|^forward " | sed "s/^/$v /"; done
