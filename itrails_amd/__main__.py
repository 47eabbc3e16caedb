"""python -m itrails_amd {optimize|viterbi|posterior} ..."""
from .cli import main

main()
