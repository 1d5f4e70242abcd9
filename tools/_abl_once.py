import sys
sys.argv=['x']
exec(open('tools/step_ablate.py').read().split("if __name__ == '__main__':")[0])
run('graph of 30', graph=30, steps=300)
