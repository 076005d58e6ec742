for v in n2 n4 n8 n2 n4 n8; do RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 200 python3 tools/enc_time.py 2>/dev/null; done
