set -o pipefail
for v in cur lw3 lw4; do for w in 1 2 4; do echo -n "$v W=$w: "; AIQMC_LIB_VARIANT=$v AIQMC_LAPW=$w timeout -k 10 120 python tools/mc_loop.py 10 N2 4096 || exit 1; done; done
for v in cur lw4; do echo -n "$v B=512 auto: "; AIQMC_LIB_VARIANT=$v timeout -k 10 120 python tools/mc_loop.py 10 N2 512 || exit 1; done
