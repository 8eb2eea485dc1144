timeout -k 10 300 python -u scratch/dbg_store2.py
