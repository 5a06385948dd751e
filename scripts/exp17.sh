#!/bin/bash
# r1 exp17: decoder layer with cross-attention key splits 1..4 (4 keys per lane), merge in the cross-out prologue
cd spittle_amd
for i in 1 2; do for xs in 1 2 3 4; do
  timeout -k 5 60 ./ubench layer 8 1 $xs > /tmp/o.txt || exit 1; sed "s/^/xsplit=$xs /" /tmp/o.txt
done; done
