set -x
ls -la /dev/dri /dev/kfd
ls /sys/class/kfd/kfd/topology/nodes | head -20
cat /sys/module/amdgpu/initstate
python3 -c "import torch; print('torch devices', torch.cuda.device_count())"
gpu_operator_amd/_native/bin/amd-node-probe | head -c 3000; echo
for f in /dev/dri/renderD*; do test -r $f -a -w $f && echo "rw $f"; done
id
