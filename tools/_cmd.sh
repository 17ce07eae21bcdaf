export TMPDIR=/tmp
timeout -k 10 400 python bench.py > /tmp/b.json 2>/tmp/b.err; rc=$?; cat /tmp/b.json; [ $rc -eq 0 ] || tail -20 /tmp/b.err
