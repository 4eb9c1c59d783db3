set -e
# MODE 1 exclusive (bit 1), MODE 0 co-resident: 32x32 tiles (~42 KB LDS) vs 32x64 (~82 KB)
GRAPHS="0 1" NCH="3" SKELDIFF_FULL_LDS=2 SKELDIFF_GL4_CFG=811 timeout -k 10 200 python -u tools/chain_debug.py 20
GRAPHS="0" NCH="3" SKELDIFF_FULL_LDS=2 SKELDIFF_GL4_CFG=811 timeout -k 10 200 python -u tools/chain_debug.py 100
GRAPHS="0 1" NCH="3" SKELDIFF_FULL_LDS=2 SKELDIFF_GL4_CFG=812 timeout -k 10 200 python -u tools/chain_debug.py 20
