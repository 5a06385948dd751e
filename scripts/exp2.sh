#!/bin/bash
R=spittle_amd/ubench_ref
T="timeout -k 5 60"
set -e
$T $R layer 8 1
$T $R layer 4 1
$T $R layer2 4 1
$T $R layer2 8 1
$T $R layer 8 1 2 8
$T $R null
