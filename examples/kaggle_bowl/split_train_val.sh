#!/bin/bash
# Split a shuffled list into a training part and a validation part.
# Usage: bash split_train_val.sh all.lst [n_train]
N=${2:-20000}
head -n "$N" "$1" > tr.lst
tail -n +"$((N + 1))" "$1" > va.lst
