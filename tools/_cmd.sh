timeout -k 10 200 python tools/ablate_res64.py
