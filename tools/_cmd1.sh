set -u
bash tools/run_variants.sh || exit $?
echo "== with MGP_ZS_WGS=512"
MGP_ZS_WGS=512 bash tools/run_variants.sh
