import struct, zipfile, sys
OPS = {0x00:('nop',0),0x01:('aconst_null',0),0x02:('iconst_m1',0),0x03:('iconst_0',0),0x04:('iconst_1',0),0x05:('iconst_2',0),0x06:('iconst_3',0),0x07:('iconst_4',0),0x08:('iconst_5',0),
0x09:('lconst_0',0),0x0a:('lconst_1',0),0x0b:('fconst_0',0),0x0c:('fconst_1',0),0x0d:('fconst_2',0),0x0e:('dconst_0',0),0x0f:('dconst_1',0),
0x10:('bipush',1),0x11:('sipush',2),0x12:('ldc',1),0x13:('ldc_w',2),0x14:('ldc2_w',2),0x15:('iload',1),0x16:('lload',1),0x17:('fload',1),0x18:('dload',1),0x19:('aload',1),
0x1a:('iload_0',0),0x1b:('iload_1',0),0x1c:('iload_2',0),0x1d:('iload_3',0),0x1e:('lload_0',0),0x1f:('lload_1',0),0x20:('lload_2',0),0x21:('lload_3',0),0x22:('fload_0',0),0x23:('fload_1',0),0x24:('fload_2',0),0x25:('fload_3',0),
0x26:('dload_0',0),0x27:('dload_1',0),0x28:('dload_2',0),0x29:('dload_3',0),0x2a:('aload_0',0),0x2b:('aload_1',0),0x2c:('aload_2',0),0x2d:('aload_3',0),
0x2e:('iaload',0),0x2f:('laload',0),0x30:('faload',0),0x31:('daload',0),0x32:('aaload',0),0x33:('baload',0),0x34:('caload',0),0x35:('saload',0),
0x36:('istore',1),0x37:('lstore',1),0x38:('fstore',1),0x39:('dstore',1),0x3a:('astore',1),0x3b:('istore_0',0),0x3c:('istore_1',0),0x3d:('istore_2',0),0x3e:('istore_3',0),
0x3f:('lstore_0',0),0x40:('lstore_1',0),0x41:('lstore_2',0),0x42:('lstore_3',0),0x43:('fstore_0',0),0x44:('fstore_1',0),0x45:('fstore_2',0),0x46:('fstore_3',0),0x47:('dstore_0',0),0x48:('dstore_1',0),0x49:('dstore_2',0),0x4a:('dstore_3',0),
0x4b:('astore_0',0),0x4c:('astore_1',0),0x4d:('astore_2',0),0x4e:('astore_3',0),0x4f:('iastore',0),0x50:('lastore',0),0x51:('fastore',0),0x52:('dastore',0),0x53:('aastore',0),0x54:('bastore',0),0x55:('castore',0),0x56:('sastore',0),
0x57:('pop',0),0x58:('pop2',0),0x59:('dup',0),0x5a:('dup_x1',0),0x5b:('dup_x2',0),0x5c:('dup2',0),0x5d:('dup2_x1',0),0x5e:('dup2_x2',0),0x5f:('swap',0),
0x60:('iadd',0),0x61:('ladd',0),0x62:('fadd',0),0x63:('dadd',0),0x64:('isub',0),0x65:('lsub',0),0x66:('fsub',0),0x67:('dsub',0),0x68:('imul',0),0x69:('lmul',0),0x6a:('fmul',0),0x6b:('dmul',0),
0x6c:('idiv',0),0x6d:('ldiv',0),0x6e:('fdiv',0),0x6f:('ddiv',0),0x70:('irem',0),0x71:('lrem',0),0x72:('frem',0),0x73:('drem',0),0x74:('ineg',0),0x75:('lneg',0),0x76:('fneg',0),0x77:('dneg',0),
0x78:('ishl',0),0x79:('lshl',0),0x7a:('ishr',0),0x7b:('lshr',0),0x7c:('iushr',0),0x7d:('lushr',0),0x7e:('iand',0),0x7f:('land',0),0x80:('ior',0),0x81:('lor',0),0x82:('ixor',0),0x83:('lxor',0),
0x84:('iinc',2),0x85:('i2l',0),0x86:('i2f',0),0x87:('i2d',0),0x88:('l2i',0),0x89:('l2f',0),0x8a:('l2d',0),0x8b:('f2i',0),0x8c:('f2l',0),0x8d:('f2d',0),0x8e:('d2i',0),0x8f:('d2l',0),0x90:('d2f',0),0x91:('i2b',0),0x92:('i2c',0),0x93:('i2s',0),
0x94:('lcmp',0),0x95:('fcmpl',0),0x96:('fcmpg',0),0x97:('dcmpl',0),0x98:('dcmpg',0),
0x99:('ifeq',2),0x9a:('ifne',2),0x9b:('iflt',2),0x9c:('ifge',2),0x9d:('ifgt',2),0x9e:('ifle',2),0x9f:('if_icmpeq',2),0xa0:('if_icmpne',2),0xa1:('if_icmplt',2),0xa2:('if_icmpge',2),0xa3:('if_icmpgt',2),0xa4:('if_icmple',2),0xa5:('if_acmpeq',2),0xa6:('if_acmpne',2),
0xa7:('goto',2),0xac:('ireturn',0),0xad:('lreturn',0),0xae:('freturn',0),0xaf:('dreturn',0),0xb0:('areturn',0),0xb1:('return',0),
0xb2:('getstatic',2),0xb3:('putstatic',2),0xb4:('getfield',2),0xb5:('putfield',2),0xb6:('invokevirtual',2),0xb7:('invokespecial',2),0xb8:('invokestatic',2),0xb9:('invokeinterface',4),
0xbb:('new',2),0xbc:('newarray',1),0xbd:('anewarray',2),0xbe:('arraylength',0),0xbf:('athrow',0),0xc0:('checkcast',2),0xc1:('instanceof',2),0xc6:('ifnull',2),0xc7:('ifnonnull',2)}
def parse(data):
    p=8; n=struct.unpack('>H',data[p:p+2])[0]; p+=2; cp=[None]
    i=1
    while i<n:
        t=data[p]; p+=1
        if t==1:
            l=struct.unpack('>H',data[p:p+2])[0]; p+=2; cp.append(('utf8',data[p:p+l].decode('utf8','replace'))); p+=l
        elif t==3: cp.append(('int',struct.unpack('>i',data[p:p+4])[0])); p+=4
        elif t==4: cp.append(('float',struct.unpack('>f',data[p:p+4])[0])); p+=4
        elif t in (5,6): cp.append(('long' if t==5 else 'double',data[p:p+8])); p+=8; cp.append(None); i+=1
        elif t in (7,8,16): cp.append((t,struct.unpack('>H',data[p:p+2])[0])); p+=2
        elif t in (9,10,11,12,18): cp.append((t,)+struct.unpack('>HH',data[p:p+4])); p+=4
        elif t==15: cp.append((t,data[p],struct.unpack('>H',data[p+1:p+3])[0])); p+=3
        else: raise Exception('tag %d'%t)
        i+=1
    p+=6; ni=struct.unpack('>H',data[p:p+2])[0]; p+=2+2*ni
    def skip_attrs(p):
        na=struct.unpack('>H',data[p:p+2])[0]; p+=2; attrs=[]
        for _ in range(na):
            nm,l=struct.unpack('>HI',data[p:p+6]); attrs.append((cp[nm][1],data[p+6:p+6+l])); p+=6+l
        return p,attrs
    nf=struct.unpack('>H',data[p:p+2])[0]; p+=2
    for _ in range(nf): p+=6; p,_a=skip_attrs(p)
    nm=struct.unpack('>H',data[p:p+2])[0]; p+=2; methods={}
    for _ in range(nm):
        acc,ni_,di=struct.unpack('>HHH',data[p:p+6]); p+=6; p,attrs=skip_attrs(p)
        for a,b in attrs:
            if a=='Code':
                cl=struct.unpack('>I',b[4:8])[0]; methods[cp[ni_][1]+cp[di][1]]=b[8:8+cl]
    return cp,methods
def name(cp,idx):
    e=cp[idx]
    if e is None: return '?'
    if e[0] in ('int','float','utf8'): return repr(e[1])
    if e[0]==7: return cp[e[1]][1]
    if e[0]==8: return 'str:'+cp[e[1]][1]
    if e[0] in (9,10,11): return name(cp,e[1])+'.'+name(cp,e[2])
    if e[0]==12: return cp[e[1]][1]+cp[e[2]][1]
    return str(e)
def dis(cp,code):
    p=0; out=[]
    while p<len(code):
        op=code[p]
        if op==0xaa or op==0xab:
            out.append((p,'switch',None)); break
        nm,l=OPS.get(op,('op%02x'%op,0))
        arg=code[p+1:p+1+l]
        s=''
        if nm in ('bipush',): s=str(struct.unpack('>b',arg)[0])
        elif nm=='sipush': s=str(struct.unpack('>h',arg)[0])
        elif nm=='ldc': s=name(cp,arg[0])
        elif nm in ('ldc_w','ldc2_w','getstatic','putstatic','getfield','putfield','invokevirtual','invokespecial','invokestatic','new','anewarray','checkcast','instanceof'): s=name(cp,struct.unpack('>H',arg[:2])[0])
        elif nm=='invokeinterface': s=name(cp,struct.unpack('>H',arg[:2])[0])
        elif l==2 and nm.startswith(('if','goto')): s='->%d'%(p+struct.unpack('>h',arg)[0])
        elif nm=='iinc': s='%d %d'%(arg[0],struct.unpack('>b',arg[1:2])[0])
        elif l==1: s=str(arg[0])
        out.append((p,nm,s)); p+=1+l
    return out
if __name__=='__main__':
    z=zipfile.ZipFile('/root/reference/lib/trove.jar')
    cls=sys.argv[1]; meths=sys.argv[2:]
    cp,m=parse(z.read(cls))
    for k in m:
        if not meths or any(k.startswith(x) for x in meths):
            print('==',k)
            for p,nm,s in dis(cp,m[k]): print('  %4d %s %s'%(p,nm,s))
