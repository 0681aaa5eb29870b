B="python bench.py --no-cpu-baseline --no-alt --steps 8"
P='import json,sys; d=json.loads(sys.stdin.readline()); print(round(d["value"]/1e6,1), "M  kernel_ms", round(d["roofline"]["kernel_ms"],2))'
for w in 12 8; do echo "wpb$w $(OLPE_WPB=$w $B | python -c "$P")"; done
