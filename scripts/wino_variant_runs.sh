set -o pipefail
for b in "$@"; do
  for shape in "16 64 64 192" "16 128 128 96" "16 256 256 48" "16 1024 1024 12" "3 70 130 13" "2 64 64 30"; do
    echo -n "$b: "; timeout -k 5 30 ./exp/wb_$b 2 $shape 20 || exit 1
  done
done
