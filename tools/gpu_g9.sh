set -o pipefail
bash tools/ab_variants.sh main occ1
