
4
z_1Placeholder*
dtype0*
shape
:
4
z_2Placeholder*
dtype0*
shape
:

outAddz_1z_2*
T0