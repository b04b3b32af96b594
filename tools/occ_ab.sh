export VSS_TILE="1:4x16,2:2x8,3:3x16,4:2x8,5:4x8,6:2x8,7:6x8,8:2x8,9:4x8,10:6x16"
for lib in build/libvss_old.so build/libvss_new.so; do
  VSS_LIBRARY=$lib timeout -k 10 120 python bench.py --no-cpu --no-host --no-ts --no-post --no-sweep --steps 400 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], [(k['layer'], round(k['ms']*1000,2), k['wg_per_cu'], k['lds_bytes']) for k in d['kernels']])" || exit 1
done
