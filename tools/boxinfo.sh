rocm-smi --showcomputepartition --showmemorypartition 2>/dev/null | grep -i -E 'partition' | head -4
rocm-smi --showmaxpower --showclocks 2>/dev/null | grep -i -E 'max graphics|sclk|mclk|power' | head -6
python3 -c "import ctypes; print('cu', open('/sys/class/kfd/kfd/topology/nodes/1/properties').read().count('simd'))" 2>/dev/null
