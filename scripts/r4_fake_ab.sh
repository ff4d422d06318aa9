set -o pipefail
OUT=gpurun_out/fake
mkdir -p $OUT
for n in base fakeaes fakedec fakecomp fakeall; do
  R=.; [ $n != base ] && R=ab/$n
  timeout -k 10 200 python scripts/ab_online.py --root $R --batch 1 --steps 20 --relu joint --detail > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
  echo "$n $(head -c 200 $OUT/$n.json)"
done
