# usage: bash tools/ab_lib.sh ALT_LIB CMD...: runs CMD with the in-tree library and with ALT_LIB (KINET_AMD_LIB), A B A B
set -e
alt=$1; shift
for i in 1 2; do
  echo "== main"; timeout -k 10 200 "$@"
  echo "== alt $alt"; KINET_AMD_LIB=$alt timeout -k 10 200 "$@"
done
