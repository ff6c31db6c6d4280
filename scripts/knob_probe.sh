cd $GRAFT_REPO_ROOT
for k in 0 256; do
  DCA_TEAM_KNOBS=$k timeout -k 10 100 python -u -c "
import sys; sys.path.insert(0,'scripts'); sys.argv=['x']
import lstm_latency as L, json
r=L.bench(8,1400,512,reps=10)
print('knobs',$k, json.dumps(r))
" || exit 1
done
