set -e
GRAPHS="0" NCH="3" SKELDIFF_FULL_LDS=0 timeout -k 10 200 python -u tools/chain_debug.py 2
GRAPHS="0" NCH="3" SKELDIFF_FULL_LDS=0 timeout -k 10 200 python -u tools/chain_debug.py 20
GRAPHS="1" NCH="3" SKELDIFF_FULL_LDS=0 timeout -k 10 200 python -u tools/chain_debug.py 20
